#!/usr/bin/env python3
"""Flagship serving benchmark (BASELINE.json metric on its config #2).

Metric: output tokens/s for the reference sizing-guide "Chatbot" use case
(third_party/IBM/docs/sizing-guide.md:56: Llama-3.1-8B-Instruct, 128 input / 128
output tokens, 65 concurrent users, 1 accelerator -> 3264 tok/s on Gaudi 3),
plus p50/p90 TTFT.  Weights are random (no checkpoints offline), prompts are
synthetic random token ids of exactly --input-len tokens, every request
generates exactly --output-len tokens (ignore_eos).  Sampling is the server
default (temperature 1.0) so the full sampler kernel runs.

One "step" = one benchmark round: all --users requests arrive together and the
round ends when the last one finishes (continuous batching inside).  W untimed
rounds, then K timed rounds bracketed by barrier + device sync.

Multi-GPU (torchrun, one rank per GPU): each group of --tp ranks is one serving
replica (default TP=1 -> N data-parallel replicas, the reference's one-pod-per-
card deployment, third_party/IBM/patterns/quickstart/run_script.sh:79-81);
per-GPU work is fixed -> weak scaling.  value = total output tokens of all
replicas / max wall time over ranks.
"""

from __future__ import annotations

import argparse
import json
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BASELINE_TOK_S = {  # third_party/IBM/docs/sizing-guide.md (Gaudi 3, vLLM 0.7.2), per replica
    ("meta-llama/Llama-3.1-8B-Instruct", 128, 128): (3264.0, 1),
    ("meta-llama/Llama-3.3-70B-Instruct", 128, 128): (1120.0, 4),
}
METRIC = "output tokens/sec (node) + p50 TTFT via OpenAI endpoint, Llama-3-8B/70B"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--users", type=int, default=65)
    ap.add_argument("--input-len", type=int, default=128)
    ap.add_argument("--output-len", type=int, default=128)
    ap.add_argument("--max-num-seqs", type=int, default=256)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--block-size", type=int, default=128)
    ap.add_argument("--gpu-memory-utilization", type=float, default=0.90)
    ap.add_argument("--temperature", type=float, default=1.0)
    ap.add_argument("--enforce-eager", action="store_true")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--verbose", action="store_true")
    return ap.parse_args()


def main() -> int:
    args = parse()
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
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if torch.cuda.is_available():
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
        device="cuda" if torch.cuda.is_available() else "cpu",
        dtype=torch.bfloat16 if torch.cuda.is_available() else torch.float32,
        seed=args.seed, enforce_eager=args.enforce_eager, served_model_name=model_id)

    t_init = time.time()
    is_driver = pstate.tp_rank() == 0
    if tp > 1 and not is_driver:
        # non-driver TP rank: replay the driver's plans until it shuts down
        from enterprise_inference_amd.engine.executor import setup_runner, worker_loop
        runner = setup_runner(cfg)
        ring = [None]
        dist.broadcast_object_list(ring, src=pstate.tp_ranks()[0], group=pstate.tp_cpu_group())
        worker_loop(runner, ring[0])
        _report(args, dist, None, rank, world)
        return 0

    from enterprise_inference_amd.engine.executor import TPExecutor, UniprocExecutor
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    if tp > 1:
        ex = TPExecutor(cfg, spawn=False)
        dist.broadcast_object_list([ex.ring_name], src=rank, group=pstate.tp_cpu_group())
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

    # barriers among replica drivers only (TP workers are busy replaying plans)
    bgroup = pstate.dp_group() if tp > 1 else None
    for w in range(args.warmup):
        one_round(f"warm{w}")
    _sync_and_barrier(torch, dist, bgroup)
    prof = None
    if os.environ.get("EIA_BENCH_CPROFILE"):      # host-side profile of the timed rounds
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    engine.phase_times.clear()
    t0 = time.time()
    tot_tokens, all_ttft, all_tpot = 0, [], []
    for s in range(args.steps):
        n, tt, tp_, dt = one_round(f"step{s}")
        tot_tokens += n
        all_ttft += tt
        all_tpot += tp_
        if args.verbose:
            print(f"[rank {rank}] round {s}: {n} tok in {dt:.3f}s -> {n / dt:.0f} tok/s, "
                  f"ttft p50 {1000 * statistics.median(tt):.1f} ms", file=sys.stderr)
    _sync_and_barrier(torch, dist, bgroup)
    elapsed = time.time() - t0
    if prof is not None:
        import pstats
        prof.disable()
        with open(os.environ["EIA_BENCH_CPROFILE"], "w") as f:
            pstats.Stats(prof, stream=f).sort_stats("tottime").print_stats(45)
    if args.verbose and engine.phase_times:
        n = max(1, engine.stats.num_steps)
        print("[rank %d] host ms/step: %s" % (rank, {k: round(1e3 * v / n, 3) for k, v in
                                                     engine.phase_times.items()}), file=sys.stderr)
    if tp > 1:
        ex.shutdown()
    local_stats = {"tokens": tot_tokens, "elapsed": elapsed, "ttft": all_ttft, "tpot": all_tpot,
                   "init_s": init_s, "steps": engine.stats.num_steps,
                   "num_blocks": engine.num_blocks}
    _report(args, dist, local_stats, rank, world)
    return 0


def _sync_and_barrier(torch, dist, group=None):
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if dist.is_initialized():
        if group is not None:
            dist.barrier(group=group)
        elif int(os.environ.get("WORLD_SIZE", "1")) > 1 and dist.get_world_size() > 1:
            from enterprise_inference_amd.parallel import state as pstate
            if pstate.tp_size() == 1:
                dist.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()


def _report(args, dist, local_stats, rank, world):
    from enterprise_inference_amd.models.catalog import resolve_name

    if dist.is_initialized():
        gathered = [None] * world
        dist.all_gather_object(gathered, local_stats)
    else:
        gathered = [local_stats]
    if rank != 0:
        return
    reps = [g for g in gathered if g is not None]
    tokens = sum(g["tokens"] for g in reps)
    elapsed = max(g["elapsed"] for g in reps)
    ttft = sorted(x for g in reps for x in g["ttft"])
    tpot = sorted(x for g in reps for x in g["tpot"])

    def pct(a, p):
        return a[min(len(a) - 1, int(p / 100.0 * len(a)))] if a else None

    value = tokens / elapsed
    model_id = resolve_name(args.model)
    base = BASELINE_TOK_S.get((model_id, args.input_len, args.output_len))
    n_replicas = max(1, world // args.tp)
    vs = None
    if base is not None:
        # published number is per replica (1 Gaudi 3 for 8B); node figure = replicas x that
        vs = value / (base[0] * n_replicas)
    total_tok_s = value * (args.input_len + args.output_len) / args.output_len
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "output tokens/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1000.0 * elapsed / max(1, args.steps), 2),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None if vs is None else round(vs, 3),
        "dtype": "bf16",
        "data": "synthetic",
        "config": {"model": model_id, "global_batch": args.users * n_replicas,
                   "seq_len": args.input_len + args.output_len,
                   "input_len": args.input_len, "output_len": args.output_len,
                   "users_per_replica": args.users,
                   "parallelism": f"dp{n_replicas}" + (f"xtp{args.tp}" if args.tp > 1 else ""),
                   "weights": "random-init", "temperature": args.temperature},
        "ttft_p50_ms": round(1000 * pct(ttft, 50), 2) if ttft else None,
        "ttft_p90_ms": round(1000 * pct(ttft, 90), 2) if ttft else None,
        "tpot_p50_ms": round(1000 * pct(tpot, 50), 3) if tpot else None,
        "total_tok_s": round(total_tok_s, 2),
        "baseline_tok_s_per_replica": None if base is None else base[0],
        "init_s": round(max(g["init_s"] for g in reps), 1),
    }
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.exit(main())
