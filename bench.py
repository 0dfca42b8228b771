#!/usr/bin/env python3
"""Flagship serving benchmark: the BASELINE.json metric, measured through the OpenAI endpoint.

Metric: output tokens/s (+ TTFT p50/p90) of the reference sizing-guide "Chatbot" use
case (third_party/IBM/docs/sizing-guide.md:56: Llama-3.1-8B-Instruct, 128 input /
128 output tokens, 65 concurrent users, one accelerator -> 3264 tok/s, TTFT p90
1300 ms on Gaudi 3), measured the way the guide does (sizing-guide.md:50-56):
concurrent streaming requests against the OpenAI-compatible server.

Per replica this process (which never touches the GPU) starts
  * the real server, ``python -m enterprise_inference_amd.entrypoints.openai.api_server``
    (API process + engine-core process + TP workers), random-init weights
    (``--load-format dummy``; no checkpoints offline), and
  * client worker processes (aiohttp) that hold the --users concurrent streams:
    streaming ``POST /v1/completions`` with exactly --input-len synthetic prompt token
    ids, ``max_tokens=--output-len``, ``ignore_eos`` (exact output length), server-default
    temperature 1.0 (the full sampler kernel runs).  TTFT = first SSE token chunk.

One "step" = one round: all --users requests arrive together, the round ends when the
last stream sent ``[DONE]``.  W untimed rounds, then K timed rounds bracketed on both
sides by ``POST /eia/sync`` (the engine core runs ``torch.cuda.synchronize()``) and a
barrier over all ranks (gloo, CPU); ms_per_step = max over ranks.  Tokens are counted
from each stream's ``usage`` chunk and checked against --output-len.

Multi-GPU (torchrun, one rank per GPU): each group of --tp ranks is one serving
replica whose first rank launches a server on those GPUs (default TP=1 -> N
data-parallel replicas, the reference's one-pod-per-card deployment,
third_party/IBM/patterns/quickstart/run_script.sh:79-81): weak scaling.
``value`` = total output tokens of all replicas / max wall time over ranks.

``--mode engine`` drives ``LLMEngine`` in-process instead (no HTTP; for kernel
profiling); its line says ``"measured_via": "engine"``.
"""

from __future__ import annotations

import argparse
import json
import os
import random
import signal
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOK_S = {  # third_party/IBM/docs/sizing-guide.md (Gaudi 3, vLLM 0.7.2), per replica
    ("meta-llama/Llama-3.1-8B-Instruct", 128, 128): (3264.0, 1),
    ("meta-llama/Llama-3.3-70B-Instruct", 128, 128): (1120.0, 4),
    ("meta-llama/Llama-3.1-405B-Instruct", 128, 128): (493.0, 8),
}
BASELINE_TTFT_P90_MS = {  # same rows (chatbot 128/128): p90 TTFT on Gaudi 3
    "meta-llama/Llama-3.1-8B-Instruct": 1300.0, "meta-llama/Llama-3.3-70B-Instruct": 613.0,
    "meta-llama/Llama-3.1-405B-Instruct": 1072.0}
METRIC = "output tokens/sec (node) + p50 TTFT via OpenAI endpoint, Llama-3-8B/70B"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", default="endpoint", choices=["endpoint", "engine"])
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--co-deploy", action="store_true",
                    help="config #5: replicas alternate --model / --co-model on disjoint GPUs")
    ap.add_argument("--co-model", default="mistralai/Mistral-7B-Instruct-v0.3")
    ap.add_argument("--users", type=int, default=65)
    ap.add_argument("--input-len", type=int, default=128)
    ap.add_argument("--output-len", type=int, default=128)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--block-size", type=int, default=128)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.90)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--client-procs", type=int, default=4,
                    help="client worker processes per replica (streams are split among them)")
    ap.add_argument("--server-args", default="", help="extra api_server flags")
    ap.add_argument("--startup-timeout", type=float, default=1500)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    ap.add_argument("--closed-loop-s", type=float, default=8.0,
                    help="endpoint mode: after the burst rounds, a closed-loop window of this "
                         "many seconds (every user resubmits on completion; 0 = off)")
    ap.add_argument("--closed-loop-warm-s", type=float, default=3.0,
                    help="closed-loop ramp before the measured window")
    ap.add_argument("--extras", default="auto", choices=["auto", "on", "off"],
                    help="after the headline, also run BASELINE config #3 (Llama-3.3-70B at "
                         "TP=N, 35 users) and at N=8 config #5 (8B + Mistral-7B co-deploy); "
                         "auto = endpoint mode with N >= 2.  Reported under extra keys, "
                         "`value` is the headline only")
    ap.add_argument("--extra-budget-s", type=float, default=900.0,
                    help="wall-clock budget for all extra configurations together")
    return ap.parse_args()


def _pct(a, p):
    return a[min(len(a) - 1, int(p / 100.0 * len(a)))] if a else None


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


# --------------------------------------------------------------------------- clients

def _client_worker(conn, url: str, model: str, max_tokens: int, temperature: float,
                   timeout: float) -> None:
    """One client process: runs its share of the concurrent streams for every round."""
    import asyncio

    import aiohttp

    async def one(session, prompt):
        body = {"model": model, "prompt": prompt, "max_tokens": max_tokens, "ignore_eos": True,
                "temperature": temperature, "stream": True,
                "stream_options": {"include_usage": True}}
        t0 = time.perf_counter()
        first = None
        usage = None
        done = False
        try:
            async with session.post(url, json=body) as r:
                if r.status != 200:
                    return (False, 0.0, 0.0, 0, f"HTTP {r.status}: {(await r.text())[:200]}")
                async for line in r.content:
                    if not line.startswith(b"data: "):
                        continue
                    if first is None and line.startswith(b'data: {"id"') and b'"text":' in line:
                        first = time.perf_counter()
                    if b'"usage"' in line:
                        usage = json.loads(line[6:])["usage"]
                    elif line.startswith(b"data: [DONE]"):
                        done = True
                        break
        except Exception as e:  # noqa: BLE001 - reported as a failed request
            return (False, 0.0, 0.0, 0, repr(e))
        t1 = time.perf_counter()
        if not done or usage is None:
            return (False, 0.0, 0.0, 0, "stream ended without usage/[DONE]")
        return (True, (first or t1) - t0, t1 - t0, int(usage["completion_tokens"]), "")

    async def closed(session, spec):
        """Closed loop: `n` users, each resubmits the moment its stream ends, until t_stop.
        Returns (wall start, ok, ttft, e2e, tokens, err) per request."""
        rng = random.Random(spec["seed"])

        async def user():
            out = []
            while time.time() < spec["t_stop"]:
                p = [rng.randrange(1000, spec["vocab"]) for _ in range(spec["input_len"])]
                t = time.time()
                out.append((t,) + await one(session, p))
            return out
        rs = await asyncio.gather(*(user() for _ in range(spec["n"])))
        return [r for u in rs for r in u]

    async def main():
        conn_limit = aiohttp.TCPConnector(limit=0, force_close=False)
        to = aiohttp.ClientTimeout(total=timeout)
        async with aiohttp.ClientSession(connector=conn_limit, timeout=to) as session:
            loop = asyncio.get_running_loop()
            while True:
                msg = await loop.run_in_executor(None, conn.recv)
                if msg is None:
                    return
                if isinstance(msg, dict):
                    conn.send(await closed(session, msg))
                    continue
                res = await asyncio.gather(*(one(session, p) for p in msg))
                conn.send(res)

    asyncio.run(main())


class ClientPool:
    def __init__(self, n: int, url: str, model: str, max_tokens: int, temperature: float,
                 timeout: float = 3600.0):
        # (the timeout bounds every request; extra configs pass their remaining budget)
        import multiprocessing as mp

        ctx = mp.get_context("spawn")
        self.conns, self.procs = [], []
        for _ in range(n):
            a, b = ctx.Pipe()
            p = ctx.Process(target=_client_worker, args=(b, url, model, max_tokens, temperature,
                                                         timeout), daemon=True)
            p.start()
            self.conns.append(a)
            self.procs.append(p)

    def round(self, prompts):
        n = len(self.conns)
        shares = [prompts[i::n] for i in range(n)]
        for c, s in zip(self.conns, shares):
            c.send(s)
        out = []
        for c in self.conns:
            out += c.recv()
        return out

    def closed_loop(self, users: int, t_stop: float, input_len: int, vocab: int, seed: int):
        """Start the closed-loop users (split over the client processes); collect() later."""
        n = len(self.conns)
        for i, c in enumerate(self.conns):
            k = users // n + (1 if i < users % n else 0)
            c.send({"n": k, "t_stop": t_stop, "input_len": input_len, "vocab": vocab,
                    "seed": seed * 131 + i})

    def collect(self):
        out = []
        for c in self.conns:
            out += c.recv()
        return out

    def close(self):
        for c in self.conns:
            try:
                c.send(None)
            except OSError:
                pass
        for p in self.procs:
            p.join(timeout=10)
            if p.is_alive():
                p.terminate()


# --------------------------------------------------------------------------- server

def _visible_devices(first: int, n: int) -> str:
    cur = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    ids = cur.split(",") if cur else [str(i) for i in range(first + n)]
    return ",".join(ids[first:first + n])


def start_server(args, first_gpu: int, port: int, log_path: str,
                 model: str = None) -> subprocess.Popen:
    # the server runs its own process groups: drop every torchrun / elastic-agent variable
    # (TORCHELASTIC_USE_AGENT_STORE would make its rank 0 wait for an agent-hosted store)
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                        "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE",
                        "MASTER_ADDR", "MASTER_PORT")
           and not k.startswith("TORCHELASTIC_")}
    env["HIP_VISIBLE_DEVICES"] = _visible_devices(first_gpu, args.tp)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env["EIA_BENCH_ENDPOINTS"] = "1"          # /eia/sync + /eia/stats (opt-in, bench only)
    cmd = [sys.executable, "-m", "enterprise_inference_amd.entrypoints.openai.api_server",
           "--model", model or args.model, "--port", str(port), "--host", "127.0.0.1",
           "--load-format", "dummy", "--tensor-parallel-size", str(args.tp),
           "--max-model-len", str(args.input_len + args.output_len + 64),
           "--max-num-seqs", str(args.max_num_seqs),
           "--max-num-batched-tokens", str(args.max_num_batched_tokens),
           "--block-size", str(args.block_size),
           "--gpu-memory-utilization", str(args.gpu_memory_utilization),
           "--seed", str(args.seed), "--disable-log-requests", "--uvicorn-log-level", "warning"]
    if args.enforce_eager:
        cmd.append("--enforce-eager")
    cmd += args.server_args.split()
    log = open(log_path, "w")
    return subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=log, stderr=subprocess.STDOUT,
                            start_new_session=True)


def _http(method: str, url: str, timeout: float = 600.0):
    import urllib.request

    req = urllib.request.Request(url, method=method, data=b"" if method == "POST" else None)
    with urllib.request.urlopen(req, timeout=timeout) as r:
        return r.status, r.read()


def wait_healthy(base: str, proc: subprocess.Popen, timeout: float, log_path: str) -> None:
    t0 = time.time()
    while time.time() - t0 < timeout:
        if proc.poll() is not None:
            tail = open(log_path).read()[-4000:]
            raise RuntimeError(f"server exited with code {proc.returncode}:\n{tail}")
        try:
            if _http("GET", base + "/health", 2.0)[0] == 200:
                return
        except Exception:  # noqa: BLE001 - not up yet
            pass
        time.sleep(0.5)
    raise TimeoutError("server did not become healthy")


def stop_server(proc: subprocess.Popen) -> None:
    if proc.poll() is None:
        os.killpg(proc.pid, signal.SIGTERM)
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            os.killpg(proc.pid, signal.SIGKILL)
            proc.wait(timeout=30)


class Replica:
    """One serving replica: an OpenAI server on GPUs [first_gpu, first_gpu + tp) plus the
    client processes holding its --users concurrent streams."""

    def __init__(self, args, idx: int, first_gpu: int, model: str, logdir: str,
                 tag: str = "", request_timeout: float = 3600.0):
        self.args, self.idx, self.model = args, idx, model
        self.log_path = os.path.join(logdir, f"bench_server{tag}_rank{first_gpu}.log")
        port = _free_port()
        self.base = f"http://127.0.0.1:{port}"
        self._closed = False
        self.proc = start_server(args, first_gpu, port, self.log_path, model)
        self.pool = ClientPool(max(1, min(args.client_procs, args.users)),
                               self.base + "/v1/completions", model, args.output_len,
                               args.temperature, request_timeout)
        from enterprise_inference_amd.models.catalog import resolve_name
        from enterprise_inference_amd.models.loader import resolve_model_config
        self.vocab = min(resolve_model_config(resolve_name(model)).vocab_size, 128000)
        self.rng = random.Random(args.seed * 7919 + first_gpu)
        self.res = []
        self.init_s = 0.0

    def wait(self) -> None:
        t0 = time.time()
        wait_healthy(self.base, self.proc, self.args.startup_timeout, self.log_path)
        self.init_s = time.time() - t0

    def one_round(self):
        a = self.args
        prompts = [[self.rng.randrange(1000, self.vocab) for _ in range(a.input_len)]
                   for _ in range(a.users)]
        return self.pool.round(prompts)

    def rounds(self, n: int, timed: bool) -> None:
        for s in range(n):
            t0 = time.time()
            res = self.one_round()
            if not timed:
                bad = [r for r in res if not r[0]]
                if bad:
                    raise RuntimeError(f"warmup request failed: {bad[0][4]}")
                continue
            self.res.append(res)
            if self.args.verbose:
                ok_tt = sorted(r[1] for r in res if r[0]) or [0.0]
                print(f"[replica {self.idx}] round {s}: {sum(r[3] for r in res)} tok in "
                      f"{time.time() - t0:.3f}s, ttft p50 {1000 * statistics.median(ok_tt):.1f} ms",
                      file=sys.stderr)

    def sync(self) -> None:
        _http("POST", self.base + "/eia/sync")

    def stats(self) -> dict:
        return json.loads(_http("GET", self.base + "/eia/stats")[1])

    def summary(self, elapsed: float, stats0: dict, stats1: dict) -> dict:
        if self.args.verbose:
            nst = max(1, stats1["num_steps"] - stats0["num_steps"])
            for key in ("phase_times", "loop_times"):
                a, b = stats0.get(key) or {}, stats1.get(key) or {}
                print(f"[replica {self.idx}] {key} ms/step: " + json.dumps(
                    {k: round(1e3 * (b[k] - a.get(k, 0.0)) / nst, 3) for k in b}),
                    file=sys.stderr)
        tot, ttft, tpot, e2e, failed = 0, [], [], [], []
        for res in self.res:
            for ok, tt, ee, n, err in res:
                if not ok or n != self.args.output_len:
                    failed.append(err or f"got {n} tokens, expected {self.args.output_len}")
                    continue
                tot += n
                ttft.append(tt)
                e2e.append(ee)
                if n > 1:
                    tpot.append((ee - tt) / (n - 1))
        return {"tokens": tot, "elapsed": elapsed, "ttft": ttft, "tpot": tpot, "e2e": e2e,
                "failed": failed, "init_s": self.init_s, "model": self.model,
                "engine_gen_tokens": stats1["num_generation_tokens"]
                - stats0["num_generation_tokens"],
                "engine_steps": stats1["num_steps"] - stats0["num_steps"],
                "engine_busy_s": stats1["step_time_s"] - stats0["step_time_s"],
                "sync_steps": stats1.get("num_sync_steps", 0) - stats0.get("num_sync_steps", 0),
                "num_blocks": stats1["num_blocks"], "dist": stats1.get("dist")}

    def closed_loop(self, dur: float, warm: float) -> dict:
        """Steady-state arrival: every user resubmits on completion.  Throughput = engine
        generation tokens over the measured window (stats read at its edges); TTFT / TPOT of
        the requests that STARTED inside the window."""
        a = self.args
        t_meas0 = time.time() + warm
        t_meas1 = t_meas0 + dur
        self.pool.closed_loop(a.users, t_meas1, a.input_len, self.vocab, a.seed + 17)
        time.sleep(max(0.0, t_meas0 - time.time()))
        s0, w0 = self.stats(), time.time()
        time.sleep(max(0.0, t_meas1 - time.time()))
        s1, w1 = self.stats(), time.time()
        res = self.pool.collect()
        inside = [r for r in res if t_meas0 <= r[0] < t_meas1]
        ok = [r for r in inside if r[1] and r[4] == a.output_len]
        return {"gen_tokens": s1["num_generation_tokens"] - s0["num_generation_tokens"],
                "window_s": w1 - w0, "ttft": [r[2] for r in ok],
                "tpot": [(r[3] - r[2]) / (r[4] - 1) for r in ok if r[4] > 1],
                "requests": len(inside), "failed": len(inside) - len(ok)}

    def close(self) -> None:
        if self._closed:
            return
        self._closed = True
        self.pool.close()
        stop_server(self.proc)


def _parallel(fns) -> None:
    """Run callables on threads, re-raise the first failure."""
    import threading

    errs = []

    def wrap(f):
        try:
            f()
        except BaseException as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    ts = [threading.Thread(target=wrap, args=(f,)) for f in fns]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    if errs:
        raise errs[0]


def replica_models(args, n: int):
    """Model of each replica: all --model, or alternating --model / --co-model (config #5,
    multi-model co-deploy on disjoint GPU sets)."""
    if not args.co_deploy:
        return [args.model] * n
    return [args.model if i % 2 == 0 else args.co_model for i in range(n)]


def run_endpoint(args) -> int:
    """Two launch forms, same measurement:
    * torchrun (RANK/WORLD_SIZE set, the driver's multi-GPU form): every --tp-th rank leads
      one replica on its GPU slice, a gloo barrier brackets the timed rounds, max over ranks;
    * fan-out (no torchrun env): this process starts --gpus / --tp replicas itself, each
      pinned to its HIP_VISIBLE_DEVICES slice, and runs their rounds concurrently."""
    if "WORLD_SIZE" in os.environ:
        return _run_endpoint_torchrun(args)
    n_rep = max(1, args.gpus // args.tp)
    if args.gpus % args.tp:
        raise SystemExit(f"--gpus {args.gpus} is not a multiple of --tp {args.tp}")
    logdir = os.environ.get("EIA_BENCH_LOGDIR") or os.path.join(ROOT, "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    models = replica_models(args, n_rep)
    reps = []
    try:
        # children first: nothing in this process ever initialises the GPU
        for i in range(n_rep):
            reps.append(Replica(args, i, i * args.tp, models[i], logdir))
        _parallel([r.wait for r in reps])
        _parallel([(lambda r=r: r.rounds(args.warmup, False)) for r in reps])
        stats0 = [r.stats() for r in reps]
        _parallel([r.sync for r in reps])
        t0 = time.time()
        _parallel([(lambda r=r: r.rounds(args.steps, True)) for r in reps])
        _parallel([r.sync for r in reps])
        elapsed = time.time() - t0
        stats1 = [r.stats() for r in reps]
        summ = [r.summary(elapsed, s0, s1) for r, s0, s1 in zip(reps, stats0, stats1)]
        closed = None
        if args.closed_loop_s > 0:
            closed = [None] * len(reps)
            _parallel([(lambda i=i, r=r: closed.__setitem__(
                i, r.closed_loop(args.closed_loop_s, args.closed_loop_warm_s)))
                for i, r in enumerate(reps)])
        for r in reps:
            r.close()
        n_gpus = n_rep * args.tp
        extras = run_extras(args, n_gpus, logdir) if want_extras(args, n_gpus) else None
        _report(args, summ, n_gpus=n_gpus, via="endpoint", closed=closed, extras=extras)
        failed = [f for g in summ for f in g["failed"]]
        if failed:
            print(f"error: {len(failed)} failed requests, e.g. {failed[0]}", file=sys.stderr)
        return 1 if failed else 0
    finally:
        for r in reps:
            r.close()


def _run_endpoint_torchrun(args) -> int:
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    leader = local % args.tp == 0
    logdir = os.environ.get("EIA_BENCH_LOGDIR") or os.path.join(ROOT, "gpurun_out")
    os.makedirs(logdir, exist_ok=True)
    rep = None
    if leader:
        model = replica_models(args, world // args.tp)[rank // args.tp]
        rep = Replica(args, rank // args.tp, local, model, logdir)
    dist = None
    if world > 1:
        import datetime

        import torch.distributed as dist
        # long timeout: the other ranks wait in a barrier while rank 0 runs the extra configs
        dist.init_process_group("gloo", rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=args.extra_budget_s + 3600))
    try:
        if rep:
            rep.wait()
            rep.rounds(args.warmup, False)
        stats0 = rep.stats() if rep else None

        def barrier():
            if rep:
                rep.sync()
            if dist is not None:
                dist.barrier()

        barrier()
        t0 = time.time()
        if rep:
            rep.rounds(args.steps, True)
            rep.sync()
        elapsed = time.time() - t0
        if dist is not None:
            dist.barrier()
        local_stats = rep.summary(elapsed, stats0, rep.stats()) if rep else None
        local_closed = None
        if rep and args.closed_loop_s > 0:
            local_closed = rep.closed_loop(args.closed_loop_s, args.closed_loop_warm_s)
        if dist is not None:
            gathered = [None] * world
            dist.all_gather_object(gathered, (local_stats, local_closed))
        else:
            gathered = [(local_stats, local_closed)]
        summ = [g[0] for g in gathered if g[0] is not None]
        closed = [g[1] for g in gathered if g[1] is not None] or None
        if rep is not None:
            rep.close()                       # free the GPUs for the extra configurations
        if dist is not None:
            dist.barrier()
        extras = None
        if rank == 0 and want_extras(args, world):
            extras = run_extras(args, world, logdir)
        if dist is not None:
            dist.barrier()
        if rank == 0:
            _report(args, summ, n_gpus=world, via="endpoint", closed=closed, extras=extras)
        failed = [f for g in summ for f in g["failed"]]
        if failed and rank == 0:
            print(f"error: {len(failed)} failed requests, e.g. {failed[0]}", file=sys.stderr)
        return 1 if failed else 0
    finally:
        if rep is not None:
            rep.close()
        if dist is not None:
            dist.destroy_process_group()


# --------------------------------------------------------------------------- extra configs

def want_extras(args, n_gpus: int) -> bool:
    if args.extras == "off" or args.mode != "endpoint":
        return False
    return args.extras == "on" or n_gpus >= 2


def _extra(a, slots, n_gpus: int, deadline: float, logdir: str) -> dict:
    """One extra configuration: replicas (first GPU, model) started, warmed, timed; any
    failure (OOM, startup error, budget exhausted) is recorded instead of raised."""
    reps = []
    try:
        left = deadline - time.time()
        if left < 120:
            return {"error": "skipped: extra budget exhausted"}
        a.startup_timeout = min(a.startup_timeout, left)
        for i, (g, m) in enumerate(slots):
            reps.append(Replica(a, i, g, m, logdir, tag="_extra",
                                request_timeout=min(300, max(60, left))))
        _parallel([r.wait for r in reps])
        _parallel([(lambda r=r: r.rounds(a.warmup, False)) for r in reps])
        stats0 = [r.stats() for r in reps]
        _parallel([r.sync for r in reps])
        t0 = time.time()
        _parallel([(lambda r=r: r.rounds(a.steps, True)) for r in reps])
        _parallel([r.sync for r in reps])
        elapsed = time.time() - t0
        stats1 = [r.stats() for r in reps]
        summ = [r.summary(elapsed, s0, s1) for r, s0, s1 in zip(reps, stats0, stats1)]
        d = _summary(a, summ, n_gpus, "endpoint")
        keep = ("value", "vs_baseline", "ms_per_step", "ttft_p50_ms", "ttft_p90_ms",
                "tpot_p50_ms", "tpot_p90_ms", "failed_requests", "init_s",
                "baseline_tok_s_per_replica", "per_model", "engine_tok_s", "dist")
        r = {k: d[k] for k in keep if k in d}
        r.update(model=d["config"]["model"], users_per_replica=a.users,
                 parallelism=d["config"]["parallelism"], steps=a.steps,
                 input_len=a.input_len, output_len=a.output_len)
        return r
    except BaseException as e:  # noqa: BLE001 - recorded, never fails the headline
        return {"error": repr(e)[-600:]}
    finally:
        for r in reps:
            try:
                r.close()
            except Exception:  # noqa: BLE001
                pass


def run_extras(args, n_gpus: int, logdir: str) -> dict:
    """BASELINE.json config #3 (Llama-3.3-70B, one replica over all N GPUs, 35 users -- the
    sizing guide's 70B row, third_party/IBM/docs/sizing-guide.md:69) and, on 8 GPUs, config #5
    (4 x Llama-3.1-8B + 4 x Mistral-7B replicas on disjoint GPUs, 65 users each)."""
    import copy
    deadline = time.time() + args.extra_budget_s
    out = {}
    a3 = copy.copy(args)
    a3.model, a3.tp, a3.users = "meta-llama/Llama-3.3-70B-Instruct", n_gpus, 35
    a3.steps, a3.warmup, a3.co_deploy = 2, 1, False
    out[f"config3_llama70b_tp{n_gpus}"] = _extra(a3, [(0, a3.model)], n_gpus, deadline, logdir)
    if n_gpus == 8:
        a5 = copy.copy(args)
        a5.tp, a5.co_deploy, a5.steps, a5.warmup = 1, True, 2, 1
        models = replica_models(a5, 8)
        out["config5_codeploy_8b_mistral7b"] = _extra(a5, list(enumerate(models)), 8, deadline,
                                                      logdir)
    return out


# --------------------------------------------------------------------------- engine mode

def run_engine(args) -> int:
    import torch
    import torch.distributed as dist

    from enterprise_inference_amd.config import (CacheConfig, EngineConfig, ParallelConfig,
                                                 SchedulerConfig)
    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    from enterprise_inference_amd.models.catalog import resolve_name
    from enterprise_inference_amd.models.loader import resolve_model_config
    from enterprise_inference_amd.parallel import state as pstate

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available()
    if gpu:
        torch.cuda.set_device(local)
    tp = args.tp
    if world > 1 or tp > 1:
        pstate.init_distributed(tp_size=tp)
    model_id = resolve_name(args.model)
    mcfg = resolve_model_config(model_id)
    cfg = EngineConfig(
        model=mcfg,
        cache=CacheConfig(block_size=args.block_size,
                          gpu_memory_utilization=args.gpu_memory_utilization),
        scheduler=SchedulerConfig(max_num_seqs=args.max_num_seqs,
                                  max_num_batched_tokens=args.max_num_batched_tokens,
                                  max_model_len=args.input_len + args.output_len + 64),
        parallel=ParallelConfig(tensor_parallel_size=tp),
        device="cuda" if gpu else "cpu", dtype=torch.bfloat16 if gpu else torch.float32,
        seed=args.seed, enforce_eager=args.enforce_eager, served_model_name=model_id,
        load_format="dummy")
    t_init = time.time()
    if tp > 1 and pstate.tp_rank() != 0:
        # non-driver TP rank: replay the driver's plans until it shuts down
        from enterprise_inference_amd.engine.executor import setup_runner, worker_loop
        runner = setup_runner(cfg)
        ring = [None, None]
        dist.broadcast_object_list(ring, src=pstate.tp_ranks()[0], group=pstate.tp_cpu_group())
        worker_loop(runner, ring[0], ring[1])
        _gather_report(args, dist, None, rank, world, via="engine")
        return 0
    from enterprise_inference_amd.engine.executor import TPExecutor, UniprocExecutor
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    if tp > 1:
        ex = TPExecutor(cfg, spawn=False)
        dist.broadcast_object_list([ex.ring_name, os.getpid()], src=rank,
                                   group=pstate.tp_cpu_group())
    else:
        ex = UniprocExecutor(cfg)
    engine = LLMEngine(cfg, executor=ex)
    init_s = time.time() - t_init
    rng = random.Random(args.seed * 7919 + rank)
    vocab = min(mcfg.vocab_size, 128000)
    params = SamplingParams(max_tokens=args.output_len, ignore_eos=True,
                            temperature=args.temperature)

    def one_round(tag: str):
        prompts = [[rng.randrange(1000, vocab) for _ in range(args.input_len)]
                   for _ in range(args.users)]
        t0 = time.time()
        for i, p in enumerate(prompts):
            engine.add_request(f"{tag}-{i}", prompt_token_ids=p, params=params, arrival_time=t0)
        ttfts, tpots, out_tokens = [], [], 0
        while engine.has_unfinished_requests():
            for o in engine.step():
                if o.finished:
                    m = o.metrics
                    n = len(o.outputs[0].token_ids)
                    out_tokens += n
                    ttfts.append(m.first_token_time - m.arrival_time)
                    if n > 1:
                        tpots.append((m.last_token_time - m.first_token_time) / (n - 1))
        return out_tokens, ttfts, tpots, time.time() - t0

    def sync_barrier():
        if gpu:
            torch.cuda.synchronize()
        if dist.is_initialized():
            if tp > 1:
                dist.barrier(group=pstate.dp_group())
            else:
                dist.barrier()
        if gpu:
            torch.cuda.synchronize()

    for w in range(args.warmup):
        one_round(f"warm{w}")
    sync_barrier()
    engine.phase_times.clear()
    t0 = time.time()
    tot_tokens, all_ttft, all_tpot = 0, [], []
    for s in range(args.steps):
        n, tt, tp_, dt = one_round(f"step{s}")
        tot_tokens += n
        all_ttft += tt
        all_tpot += tp_
    sync_barrier()
    elapsed = time.time() - t0
    if args.verbose and engine.phase_times:
        n = max(1, engine.stats.num_steps)
        print("[rank %d] host ms/step: %s" % (rank, {k: round(1e3 * v / n, 3) for k, v in
                                                     engine.phase_times.items()}), file=sys.stderr)
    if tp > 1:
        ex.shutdown()
    local_stats = {"tokens": tot_tokens, "elapsed": elapsed, "ttft": all_ttft, "tpot": all_tpot,
                   "e2e": [], "failed": [], "init_s": init_s, "num_blocks": engine.num_blocks,
                   "model": model_id, "dist": ex.dist_info()}
    _gather_report(args, dist, local_stats, rank, world, via="engine")
    return 0


# --------------------------------------------------------------------------- report

def dist_summary(ranks) -> dict:
    """Compact self-description of one replica from its ranks' ``describe_distributed``
    records (engine/executor.py): the world size each rank's process group formed, the
    collective backend, and the custom all-reduce decision (active / reason / thresholds /
    per-size timings) -- identical on every rank by construction, checked here."""
    ranks = [r for r in (ranks or []) if isinstance(r, dict) and "error" not in r]
    if not ranks:
        return {"ranks": 0}
    ar = [r.get("custom_allreduce") or {} for r in ranks]
    out = {"ranks": len(ranks), "tp": ranks[0].get("tp_size", 1),
           "pp": ranks[0].get("pp_size", 1),
           "world_sizes": [r.get("world_size") for r in ranks],
           "backend": ranks[0].get("backend")}
    if out["tp"] > 1 or out["pp"] > 1:
        out["custom_allreduce"] = ar[0]
        out["custom_allreduce_agreed"] = all(
            (a.get("active"), a.get("oneshot_max"), a.get("use_max")) ==
            (ar[0].get("active"), ar[0].get("oneshot_max"), ar[0].get("use_max")) for a in ar)
    return out


def _gather_report(args, dist, local_stats, rank, world, via: str):
    if dist is not None and dist.is_initialized():
        gathered = [None] * world
        dist.all_gather_object(gathered, local_stats)
    else:
        gathered = [local_stats]
    if rank == 0:
        _report(args, [g for g in gathered if g is not None], world, via)


def _report(args, reps, n_gpus: int, via: str, closed=None, extras=None):
    """ONE JSON line for the whole job: ``reps`` holds one summary per serving replica."""
    out = _summary(args, reps, n_gpus, via)
    if closed:
        tt = sorted(x for c in closed for x in c["ttft"])
        tp = sorted(x for c in closed for x in c["tpot"])
        out["closed_loop"] = {
            "tok_s": round(sum(c["gen_tokens"] / max(c["window_s"], 1e-9) for c in closed), 2),
            "window_s": round(max(c["window_s"] for c in closed), 2),
            "users_per_replica": args.users,
            "requests": sum(c["requests"] for c in closed),
            "failed_requests": sum(c["failed"] for c in closed),
            "ttft_p50_ms": None if not tt else round(1000 * _pct(tt, 50), 2),
            "ttft_p90_ms": None if not tt else round(1000 * _pct(tt, 90), 2),
            "tpot_p50_ms": None if not tp else round(1000 * _pct(tp, 50), 3),
            "tpot_p90_ms": None if not tp else round(1000 * _pct(tp, 90), 3)}
    if extras is not None:
        out["extra_configs"] = extras
    print(json.dumps(out), flush=True)


def _summary(args, reps, n_gpus: int, via: str) -> dict:
    from enterprise_inference_amd.models.catalog import resolve_name

    tokens = sum(g["tokens"] for g in reps)
    elapsed = max(g["elapsed"] for g in reps)
    ttft = sorted(x for g in reps for x in g["ttft"])
    tpot = sorted(x for g in reps for x in g["tpot"])
    e2e = sorted(x for g in reps for x in g["e2e"])
    value = tokens / elapsed
    n_replicas = len(reps)
    models = [resolve_name(g.get("model") or args.model) for g in reps]
    # published numbers are per replica (e.g. 1 Gaudi 3 for 8B): node = sum over replicas;
    # null when any replica's model has no published number (Mistral-7B, Mixtral)
    bases = [BASELINE_TOK_S.get((m, args.input_len, args.output_len)) for m in models]
    vs = value / sum(b[0] for b in bases) if all(b is not None for b in bases) else None
    base = bases[0]

    def ms(v, nd=2):
        return None if v is None else round(1000 * v, nd)

    uniq = list(dict.fromkeys(models))
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "output tokens/s",
        "n_gpus": n_gpus,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / max(1, args.steps), 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None if vs is None else round(vs, 3),
        "dtype": "bf16",
        "data": "synthetic",
        "config": {"model": "+".join(uniq), "global_batch": args.users * n_replicas,
                   "seq_len": args.input_len + args.output_len,
                   "input_len": args.input_len, "output_len": args.output_len,
                   "users_per_replica": args.users,
                   "parallelism": f"dp{n_replicas}" + (f"xtp{args.tp}" if args.tp > 1 else ""),
                   "weights": "random-init", "temperature": args.temperature},
        "measured_via": via,
        "ttft_p50_ms": ms(_pct(ttft, 50)),
        "ttft_p90_ms": ms(_pct(ttft, 90)),
        "tpot_p50_ms": ms(_pct(tpot, 50), 3),
        "tpot_p90_ms": ms(_pct(tpot, 90), 3),
        "e2e_p50_ms": ms(_pct(e2e, 50)),
        "total_tok_s": round(value * (args.input_len + args.output_len) / args.output_len, 2),
        "baseline_tok_s_per_replica": None if base is None else base[0],
        "baseline_ttft_p90_ms_gaudi3": None if base is None else
        BASELINE_TTFT_P90_MS.get(models[0]),
        "failed_requests": sum(len(g["failed"]) for g in reps),
        "init_s": round(max(g["init_s"] for g in reps), 1),
    }
    if len(uniq) > 1:
        out["per_model"] = {m: {"tok_s": round(sum(g["tokens"] for g, mm in zip(reps, models)
                                                  if mm == m) / elapsed, 2),
                                "replicas": models.count(m)} for m in uniq}
    ds = [dist_summary(g.get("dist")) for g in reps if g.get("dist") is not None]
    if ds:
        # one entry per replica; replicas that look the same collapse into one with a count
        uniq_d = []
        for d in ds:
            for u in uniq_d:
                if u["desc"] == d:
                    u["replicas"] += 1
                    break
            else:
                uniq_d.append({"desc": d, "replicas": 1})
        out["dist"] = [dict(u["desc"], replicas=u["replicas"]) for u in uniq_d]
    if via == "endpoint":
        busy = max(g["engine_busy_s"] for g in reps)
        # engine-level throughput over each engine core's busy time (no HTTP / client), and
        # the fraction of the timed window the engine loops were stepping
        out["engine_tok_s"] = round(sum(g["engine_gen_tokens"] / max(g["engine_busy_s"], 1e-9)
                                        for g in reps), 2)
        out["engine_busy_frac"] = round(busy / elapsed, 3)
        out["engine_steps"] = sum(g["engine_steps"] for g in reps)
        # steps that could not be launched ahead of the previous step's token read-back
        out["engine_sync_steps"] = sum(g.get("sync_steps", 0) for g in reps)
    return out


def main() -> int:
    args = parse()
    if args.mode == "engine":
        return run_engine(args)
    return run_endpoint(args)


if __name__ == "__main__":
    sys.exit(main())
