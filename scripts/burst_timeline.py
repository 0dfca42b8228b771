#!/usr/bin/env python3
"""Host timeline of one headline burst round in the engine (where the TTFT goes).

Runs the bench's engine-mode round (65 users x 128/128, Llama-3.1-8B, random-init weights)
in-process, once to warm up and once traced, and prints per engine.step() call: wall time
at entry / exit relative to the round start, the scheduled composition (prefill tokens,
prefill sequences, decodes), and the host phase deltas (schedule / launch / process incl. the
wait for the previous step's GPU result / emit).  Then the TTFT distribution and the time of
the first and last first-token.

  python scripts/burst_timeline.py --model llama-8b --users 65 --out gpurun_out/burst.md
"""
from __future__ import annotations

import argparse
import os
import random
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--users", type=int, default=65)
    ap.add_argument("--input-len", type=int, default=128)
    ap.add_argument("--output-len", type=int, default=128)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--steps-shown", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()

    import torch

    from enterprise_inference_amd.config import (CacheConfig, EngineConfig, ParallelConfig,
                                                 SchedulerConfig)
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    from enterprise_inference_amd.models.catalog import resolve_name
    from enterprise_inference_amd.models.loader import resolve_model_config

    gpu = torch.cuda.is_available()
    model_id = resolve_name(a.model)
    mcfg = resolve_model_config(model_id)
    cfg = EngineConfig(
        model=mcfg, cache=CacheConfig(block_size=128, gpu_memory_utilization=0.9),
        scheduler=SchedulerConfig(max_num_seqs=256, max_num_batched_tokens=a.max_num_batched_tokens,
                                  max_model_len=a.input_len + a.output_len + 64),
        parallel=ParallelConfig(tensor_parallel_size=1),
        device="cuda" if gpu else "cpu", dtype=torch.bfloat16 if gpu else torch.float32,
        seed=0, served_model_name=model_id, load_format="dummy")
    engine = LLMEngine(cfg)
    rng = random.Random(0)
    vocab = min(mcfg.vocab_size, 128000)
    params = SamplingParams(max_tokens=a.output_len, ignore_eos=True, temperature=1.0)

    rows = []
    orig_schedule = engine.scheduler.schedule

    def schedule():
        out = orig_schedule()
        rows.append({"npf": len(out.prefills), "pft": sum(p.num_tokens for p in out.prefills),
                     "nd": len(out.decodes)})
        return out

    engine.scheduler.schedule = schedule

    def one_round(tag: str, trace: bool):
        prompts = [[rng.randrange(1000, vocab) for _ in range(a.input_len)] for _ in range(a.users)]
        rows.clear()
        steps = []
        t0 = time.time()
        for i, p in enumerate(prompts):
            engine.add_request(f"{tag}-{i}", prompt_token_ids=p, params=params, arrival_time=t0)
        t_added = time.time() - t0
        firsts, ttfts = [], []
        while engine.has_unfinished_requests():
            pt0 = dict(engine.phase_times)
            ts = time.time() - t0
            outs = engine.step()
            te = time.time() - t0
            pt1 = engine.phase_times
            steps.append((ts, te, {k: pt1.get(k, 0.0) - pt0.get(k, 0.0) for k in pt1}))
            for o in outs:
                if o.finished:
                    m = o.metrics
                    ttfts.append(m.first_token_time - m.arrival_time)
                    firsts.append(m.first_token_time - t0)
        return t_added, steps, list(rows), ttfts, firsts, time.time() - t0

    one_round("warm", False)
    if gpu:
        torch.cuda.synchronize()
    time.sleep(0.1)   # an idle gap that marks the traced round in a kernel trace (trace_gaps.py)
    t_added, steps, comp, ttfts, firsts, total = one_round("traced", True)
    lines = [f"# Burst round timeline ({model_id}, {a.users} users x {a.input_len}/{a.output_len}, "
             f"max_num_batched_tokens {a.max_num_batched_tokens})", "",
             f"requests added in {1e3 * t_added:.2f} ms; round {1e3 * total:.1f} ms; "
             f"TTFT p50 {1e3 * statistics.median(ttfts):.1f} ms, min {1e3 * min(ttfts):.1f}, "
             f"max {1e3 * max(ttfts):.1f}; first tokens at {1e3 * min(firsts):.1f}..{1e3 * max(firsts):.1f} ms",
             "", "| step | enter ms | exit ms | prefill seqs | prefill tok | decodes | schedule | launch "
             "| process (wait) | update | emit |", "|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|---:|"]
    for i, (ts, te, d) in enumerate(steps[:a.steps_shown]):
        c = comp[i] if i < len(comp) else {"npf": 0, "pft": 0, "nd": 0}
        f = lambda k: f"{1e3 * d.get(k, 0.0):.2f}"  # noqa: E731
        lines.append(f"| {i} | {1e3 * ts:.2f} | {1e3 * te:.2f} | {c['npf']} | {c['pft']} | {c['nd']} | "
                     f"{f('schedule')} | {f('launch')} | {f('process')} ({f('wait')}) | {f('update')} | "
                     f"{f('emit')} |")
    tail = steps[a.steps_shown:]
    if tail:
        dt = [te - ts for ts, te, _ in tail]
        lines.append("")
        lines.append(f"remaining {len(tail)} steps: median {1e3 * statistics.median(dt):.2f} ms per "
                     f"step() call, last exit {1e3 * tail[-1][1]:.1f} ms")
    text = "\n".join(lines) + "\n"
    print(text, flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
