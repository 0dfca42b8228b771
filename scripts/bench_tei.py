#!/usr/bin/env python3
"""TEI embedding / rerank throughput through the HTTP server.

Starts ``enterprise_inference_amd.entrypoints.tei.server`` (random-init weights of the real
architecture, ``--load-format dummy``) for bge-base-en-v1.5 (``/v1/embeddings``) and
bge-reranker-base (``/rerank``) -- the reference's ``tei`` / ``teirerank`` catalog entries
(core/playbooks/deploy-inference-models.yml:1512-1680) -- and drives each with closed-loop
clients: every client sends its next request when the previous one returns.

Per case it prints one JSON line: requests/s, documents/s, tokens/s and the p50 / p90 request
latency over the timed window.  Documents are synthetic text of ~``--doc-tokens`` tokens (the
byte-level tokenizer of a dummy-weight model: one token per character).

  python scripts/bench_tei.py --window 10 --out gpurun_out/tei.md
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def start_server(model: str, port: int, max_batch_tokens: int):
    env = dict(os.environ, PYTHONPATH=ROOT + os.pathsep + os.environ.get("PYTHONPATH", ""))
    cmd = [sys.executable, "-m", "enterprise_inference_amd.entrypoints.tei.server",
           "--model-id", model, "--port", str(port), "--hostname", "127.0.0.1",
           "--load-format", "dummy", "--auto-truncate",
           "--max-batch-tokens", str(max_batch_tokens)]
    log = open(os.path.join(ROOT, "gpurun_out", f"tei_server_{port}.log"), "w")
    proc = subprocess.Popen(cmd, env=env, stdout=log, stderr=subprocess.STDOUT, cwd=ROOT)
    import httpx
    t0 = time.time()
    while time.time() - t0 < 600:
        if proc.poll() is not None:
            raise RuntimeError(f"TEI server exited ({proc.returncode}); see {log.name}")
        try:
            if httpx.get(f"http://127.0.0.1:{port}/health", timeout=2).status_code == 200:
                return proc
        except Exception:   # noqa: BLE001
            pass
        time.sleep(1)
    proc.kill()
    raise RuntimeError("TEI server did not become healthy")


def doc(i: int, n: int) -> str:
    base = f"passage {i}: the quick brown fox jumps over the lazy dog while the MI355X streams. "
    return (base * (n // len(base) + 1))[:n]


async def closed_loop(url: str, make_body, clients: int, window: float, warm: float):
    import httpx
    lat, done_docs, done_tok, reqs = [], [0], [0], [0]
    t_start = time.time() + warm
    t_end = t_start + window

    async def client(cid: int):
        k = 0
        async with httpx.AsyncClient(timeout=120) as c:
            while time.time() < t_end:
                body, ndocs, ntok = make_body(cid, k)
                k += 1
                t0 = time.time()
                r = await c.post(url, json=body)
                t1 = time.time()
                r.raise_for_status()
                if t0 >= t_start and t1 <= t_end:
                    lat.append(t1 - t0)
                    reqs[0] += 1
                    done_docs[0] += ndocs
                    done_tok[0] += ntok
    await asyncio.gather(*(client(i) for i in range(clients)))
    lat.sort()

    def pct(p):
        return round(1e3 * lat[min(len(lat) - 1, int(p * len(lat)))], 1) if lat else None
    return {"requests_per_s": round(reqs[0] / window, 1), "docs_per_s": round(done_docs[0] / window, 1),
            "tokens_per_s": round(done_tok[0] / window), "p50_ms": pct(0.5), "p90_ms": pct(0.9),
            "requests": reqs[0]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--window", type=float, default=10.0)
    ap.add_argument("--warm", type=float, default=3.0)
    ap.add_argument("--doc-tokens", type=int, default=510)
    ap.add_argument("--max-batch-tokens", type=int, default=16384)
    ap.add_argument("--embed-model", default="BAAI/bge-base-en-v1.5")
    ap.add_argument("--rerank-model", default="BAAI/bge-reranker-base")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    rows = []
    n = a.doc_tokens
    # (model, route, clients, docs per request)
    cases = [(a.embed_model, "/v1/embeddings", 64, 1), (a.embed_model, "/v1/embeddings", 16, 32),
             (a.embed_model, "/embed", 64, 1),
             (a.rerank_model, "/rerank", 32, 16), (a.rerank_model, "/rerank", 8, 64)]
    servers = {}
    try:
        for model, route, clients, per in cases:
            if model not in servers:
                port = _port()
                servers[model] = (start_server(model, port, a.max_batch_tokens), port)
            port = servers[model][1]
            url = f"http://127.0.0.1:{port}{route}"
            if route == "/rerank":
                qlen = 32

                def body(cid, k, per=per):
                    return ({"query": doc(10_000 + cid, qlen),
                             "texts": [doc(cid * 1000 + k * per + j, n - qlen) for j in range(per)]},
                            per, per * n)
            elif route == "/embed":
                def body(cid, k, per=per):
                    return ({"inputs": [doc(cid * 1000 + k * per + j, n) for j in range(per)]},
                            per, per * n)
            else:
                def body(cid, k, per=per, model=model):
                    return ({"model": model,
                             "input": [doc(cid * 1000 + k * per + j, n) for j in range(per)]},
                            per, per * n)
            r = asyncio.run(closed_loop(url, body, clients, a.window, a.warm))
            r.update(model=model, route=route, clients=clients, docs_per_request=per,
                     doc_tokens=n, max_batch_tokens=a.max_batch_tokens)
            rows.append(r)
            print(json.dumps(r), flush=True)
    finally:
        for proc, _ in servers.values():
            proc.terminate()
            try:
                proc.wait(30)
            except subprocess.TimeoutExpired:
                proc.kill()
    if a.out:
        with open(a.out, "w") as f:
            f.write("# TEI throughput (closed loop, random-init weights, byte tokenizer)\n\n")
            f.write("| model | route | clients | docs/req | req/s | docs/s | tokens/s | p50 ms | p90 ms |\n")
            f.write("|---|---|---:|---:|---:|---:|---:|---:|---:|\n")
            for r in rows:
                f.write(f"| {r['model']} | {r['route']} | {r['clients']} | {r['docs_per_request']} | "
                        f"{r['requests_per_s']} | {r['docs_per_s']} | {r['tokens_per_s']} | "
                        f"{r['p50_ms']} | {r['p90_ms']} |\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
