#!/usr/bin/env python3
"""OpenAI-endpoint load generator for the reference sizing-guide use cases.

The reference's only published numbers (third_party/IBM/docs/sizing-guide.md:46-89)
are per-use-case "sweet spots": fixed input/output lengths per user, N concurrent
users, output tokens/s and TTFT p90.  This client reproduces that protocol against
any OpenAI-compatible server (ours, or a vLLM pod behind APISIX / LiteLLM):

  * every user sends streaming ``/v1/completions`` requests with a synthetic prompt
    of exactly ``input_len`` token ids, ``max_tokens=output_len`` and
    ``ignore_eos=true`` (exact output length), and starts its next request as soon
    as the previous one finishes (closed loop, ``--rounds`` requests per user);
  * TTFT = time to the first streamed token, TPOT = (E2E - TTFT) / (n - 1); reports
    p50/p90/p99 and output / total tokens/s over the wall time of the timed rounds.

Without ``--base-url`` it launches our server in a child process with random-init
weights (``--load-format dummy``) and waits for ``/health``.  Examples::

  python benchmarks/serving_bench.py --use-case chatbot                 # 8B, 65 users
  python benchmarks/serving_bench.py --base-url https://host/Llama-3.1-8B-Instruct \\
      --token "$TOKEN" --use-case summarize
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import signal
import subprocess
import sys
import time
from dataclasses import dataclass
from typing import Dict, List, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# sizing-guide.md:56-63 (Llama-3.1-8B-Instruct, 1x Gaudi 3):
#   use case -> (input len, output len, users, published tok/s, published TTFT p90 ms)
USE_CASES: Dict[str, tuple] = {
    "chatbot": (128, 128, 65, 3264.0, 1300.0),
    "content-creation": (128, 2048, 35, 3172.0, 394.0),
    "code-generation": (128, 4096, 35, 2799.0, 474.0),
    "describe": (2048, 128, 210, 1318.0, 19463.0),
    "suggest": (4096, 128, 135, 800.0, 18745.0),
    "summarize": (8192, 128, 65, 391.0, 18412.0),
    "translate": (1024, 1024, 65, 2854.0, 11815.0),
    "correct": (2048, 2048, 35, 2463.0, 1921.0),
}


@dataclass
class Result:
    ok: bool
    ttft: float = 0.0
    e2e: float = 0.0
    out_tokens: int = 0
    in_tokens: int = 0
    error: str = ""


def pct(a: List[float], p: float) -> Optional[float]:
    if not a:
        return None
    s = sorted(a)
    return s[min(len(s) - 1, int(p / 100.0 * len(s)))]


async def one_request(client, url: str, headers: dict, model: str, prompt: List[int],
                      max_tokens: int, temperature: float) -> Result:
    body = {"model": model, "prompt": prompt, "max_tokens": max_tokens, "ignore_eos": True,
            "temperature": temperature, "stream": True,
            "stream_options": {"include_usage": True}}
    t0 = time.perf_counter()
    first = None
    n_chunks = 0
    usage = None
    try:
        async with client.stream("POST", url, json=body, headers=headers) as r:
            if r.status_code != 200:
                txt = (await r.aread()).decode(errors="replace")
                return Result(False, error=f"HTTP {r.status_code}: {txt[:200]}")
            async for line in r.aiter_lines():
                if not line.startswith("data:"):
                    continue
                data = line[5:].strip()
                if data == "[DONE]":
                    break
                chunk = json.loads(data)
                if chunk.get("usage"):
                    usage = chunk["usage"]
                ch = chunk.get("choices") or []
                if ch and ch[0].get("text"):
                    if first is None:
                        first = time.perf_counter()
                    n_chunks += 1
    except Exception as e:  # noqa: BLE001 - counted as a failed request
        return Result(False, error=repr(e))
    t1 = time.perf_counter()
    out = usage.get("completion_tokens", n_chunks) if usage else n_chunks
    inp = usage.get("prompt_tokens", len(prompt)) if usage else len(prompt)
    return Result(True, ttft=(first or t1) - t0, e2e=t1 - t0, out_tokens=out, in_tokens=inp)


async def run_load(base_url: str, model: str, input_len: int, output_len: int, users: int,
                   rounds: int, temperature: float, token: Optional[str], vocab: int,
                   seed: int, timeout: float) -> dict:
    import httpx

    url = base_url.rstrip("/") + "/v1/completions"
    headers = {"Authorization": f"Bearer {token}"} if token else {}
    rng = random.Random(seed)
    results: List[Result] = []
    limits = httpx.Limits(max_connections=users + 8, max_keepalive_connections=users + 8)
    async with httpx.AsyncClient(timeout=timeout, limits=limits, verify=False) as client:
        async def user(_: int):
            for _r in range(rounds):
                prompt = [rng.randrange(1000, vocab) for _ in range(input_len)]
                results.append(await one_request(client, url, headers, model, prompt,
                                                 output_len, temperature))

        t0 = time.perf_counter()
        await asyncio.gather(*(user(u) for u in range(users)))
        wall = time.perf_counter() - t0
    ok = [r for r in results if r.ok]
    out_tok = sum(r.out_tokens for r in ok)
    in_tok = sum(r.in_tokens for r in ok)
    tpot = [(r.e2e - r.ttft) / (r.out_tokens - 1) for r in ok if r.out_tokens > 1]

    def ms(v):
        return None if v is None else round(1000 * v, 2)

    return {
        "requests": len(results), "failed": len(results) - len(ok),
        "errors": sorted({r.error for r in results if not r.ok})[:5],
        "wall_s": round(wall, 3),
        "output_tok_s": round(out_tok / wall, 2) if wall > 0 else 0.0,
        "total_tok_s": round((out_tok + in_tok) / wall, 2) if wall > 0 else 0.0,
        "ttft_p50_ms": ms(pct([r.ttft for r in ok], 50)),
        "ttft_p90_ms": ms(pct([r.ttft for r in ok], 90)),
        "ttft_p99_ms": ms(pct([r.ttft for r in ok], 99)),
        "tpot_p50_ms": ms(pct(tpot, 50)), "tpot_p90_ms": ms(pct(tpot, 90)),
        "e2e_p50_ms": ms(pct([r.e2e for r in ok], 50)),
    }


def wait_health(base_url: str, proc: subprocess.Popen, timeout: float) -> None:
    import httpx

    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            raise RuntimeError(f"server exited with code {proc.returncode}")
        try:
            if httpx.get(base_url.rstrip("/") + "/health", timeout=2).status_code == 200:
                return
        except Exception:  # noqa: BLE001 - not up yet
            pass
        time.sleep(1.0)
    raise TimeoutError("server did not become healthy")


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="OpenAI-endpoint load generator (sizing-guide use cases)")
    ap.add_argument("--use-case", default="chatbot", choices=sorted(USE_CASES))
    ap.add_argument("--base-url", default=None, help="existing server (default: launch ours)")
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--token", default=os.environ.get("OPENAI_API_KEY"))
    ap.add_argument("--input-len", type=int, default=None)
    ap.add_argument("--output-len", type=int, default=None)
    ap.add_argument("--users", type=int, default=None)
    ap.add_argument("--rounds", type=int, default=2, help="requests per user (closed loop)")
    ap.add_argument("--warmup-rounds", type=int, default=1)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--vocab", type=int, default=128000)
    ap.add_argument("--port", type=int, default=2080)
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--server-args", default="", help="extra args for the launched server")
    ap.add_argument("--startup-timeout", type=float, default=900)
    ap.add_argument("--request-timeout", type=float, default=1800)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--out", default=None, help="append the JSON result line to this file")
    args = ap.parse_args(argv)

    i_len, o_len, users, pub_tok_s, pub_ttft = USE_CASES[args.use_case]
    i_len = args.input_len or i_len
    o_len = args.output_len or o_len
    users = args.users or users

    proc = None
    base = args.base_url
    if base is None:
        base = f"http://127.0.0.1:{args.port}"
        cmd = [sys.executable, "-m", "enterprise_inference_amd.entrypoints.openai.api_server",
               "--model", args.model, "--port", str(args.port), "--host", "127.0.0.1",
               "--load-format", "dummy", "--tensor-parallel-size", str(args.tp),
               "--max-model-len", str(i_len + o_len + 64), "--disable-log-requests",
               "--uvicorn-log-level", "warning"] + args.server_args.split()
        proc = subprocess.Popen(cmd, cwd=ROOT, start_new_session=True)
    try:
        if proc is not None:
            wait_health(base, proc, args.startup_timeout)
        common = dict(base_url=base, model=args.model, input_len=i_len, output_len=o_len,
                      users=users, temperature=args.temperature, token=args.token,
                      vocab=args.vocab, timeout=args.request_timeout)
        if args.warmup_rounds:
            asyncio.run(run_load(rounds=args.warmup_rounds, seed=args.seed + 1, **common))
        res = asyncio.run(run_load(rounds=args.rounds, seed=args.seed, **common))
    finally:
        if proc is not None and proc.poll() is None:
            os.killpg(proc.pid, signal.SIGTERM)
            try:
                proc.wait(timeout=60)
            except subprocess.TimeoutExpired:
                os.killpg(proc.pid, signal.SIGKILL)
    res.update({"use_case": args.use_case, "model": args.model, "input_len": i_len,
                "output_len": o_len, "users": users, "rounds": args.rounds,
                "published_tok_s_gaudi3": pub_tok_s, "published_ttft_p90_ms_gaudi3": pub_ttft})
    if "8B" in args.model:
        res["vs_published"] = round(res["output_tok_s"] / pub_tok_s, 3)
    line = json.dumps(res)
    print(line, flush=True)
    if args.out:
        with open(args.out, "a") as f:
            f.write(line + "\n")
    return 0 if res["failed"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
