#!/usr/bin/env python3
"""Where a burst round's time to first token goes (engine loop, no HTTP).

Builds the bench's engine (random-init weights of --model), runs warm-up rounds, then one burst
round of --users prompts while recording, per ``engine.step()`` call: wall-clock start / end
relative to the round's arrival time, the engine's host phase times (schedule / launch /
process / wait / update / emit, ``LLMEngine.phase_times``), the step's prefill tokens and decode
rows, and how many requests got their first token in it.  ``--tiny`` runs a small Llama on the
CPU (checks the script, not the numbers).

  python scripts/ttft_anatomy.py --model meta-llama/Llama-3.1-8B-Instruct --users 65
"""
import argparse
import json
import os
import random
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def build_engine(a):
    import torch

    from enterprise_inference_amd.config import (CacheConfig, EngineConfig, ModelConfig,
                                                 SchedulerConfig)
    from enterprise_inference_amd.engine.llm_engine import LLMEngine
    gpu = torch.cuda.is_available()
    if a.tiny:
        from enterprise_inference_amd.models.catalog import tiny_config
        mcfg = ModelConfig.from_hf_dict(tiny_config())
    else:
        from enterprise_inference_amd.models.catalog import resolve_name
        from enterprise_inference_amd.models.loader import resolve_model_config
        mcfg = resolve_model_config(resolve_name(a.model))
    cfg = EngineConfig(
        model=mcfg,
        cache=CacheConfig(block_size=a.block_size,
                          **({"num_gpu_blocks": 256} if a.tiny else {})),
        scheduler=SchedulerConfig(max_num_seqs=256, max_num_batched_tokens=a.max_num_batched_tokens,
                                  max_model_len=a.input_len + a.output_len + 64),
        device="cuda" if gpu else "cpu", dtype=torch.bfloat16 if gpu else torch.float32,
        seed=0, load_format="dummy")
    return LLMEngine(cfg), (min(mcfg.vocab_size, 128000))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="meta-llama/Llama-3.1-8B-Instruct")
    ap.add_argument("--tiny", action="store_true")
    ap.add_argument("--users", type=int, default=65)
    ap.add_argument("--input-len", type=int, default=128)
    ap.add_argument("--output-len", type=int, default=128)
    ap.add_argument("--block-size", type=int, default=128)
    ap.add_argument("--max-num-batched-tokens", type=int, default=8192)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--steps-shown", type=int, default=5)
    a = ap.parse_args()
    import torch

    from enterprise_inference_amd.engine.sampling_params import SamplingParams
    eng, vocab = build_engine(a)
    rng = random.Random(1)
    params = SamplingParams(max_tokens=a.output_len, ignore_eos=True, temperature=1.0)

    def one_round(tag, trace):
        prompts = [[rng.randrange(min(1000, vocab // 2), vocab) for _ in range(a.input_len)]
                   for _ in range(a.users)]
        t0 = time.time()
        for i, p in enumerate(prompts):
            eng.add_request(f"{tag}-{i}", prompt_token_ids=p, params=params, arrival_time=t0)
        t_add = time.time() - t0
        firsts, k = [], 0
        seen = set()
        while eng.has_unfinished_requests():
            before = dict(eng.phase_times)
            sched_before = eng.stats.num_prompt_tokens
            ts = time.time() - t0
            outs = eng.step()
            te = time.time() - t0
            new_first = 0
            for o in outs:
                if o.request_id not in seen and o.outputs and o.outputs[0].token_ids:
                    seen.add(o.request_id)
                    new_first += 1
            if trace is not None and k < a.steps_shown:
                ph = {n: round(1e3 * (v - before.get(n, 0.0)), 3)
                      for n, v in eng.phase_times.items() if v - before.get(n, 0.0) > 0}
                trace.append({"step": k, "start_ms": round(1e3 * ts, 2), "end_ms": round(1e3 * te, 2),
                              "prompt_tokens": eng.stats.num_prompt_tokens - sched_before,
                              "first_tokens": new_first, "phases_ms": ph})
            firsts += [te] * new_first
            k += 1
        firsts.sort()
        return t_add, firsts

    for w in range(a.warmup):
        one_round(f"w{w}", None)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    trace = []
    t_add, firsts = one_round("m", trace)
    print(json.dumps({"add_requests_ms": round(1e3 * t_add, 2),
                      "ttft_p50_ms": round(1e3 * firsts[len(firsts) // 2], 2),
                      "ttft_max_ms": round(1e3 * firsts[-1], 2)}))
    for t in trace:
        print(json.dumps(t))
    return 0


if __name__ == "__main__":
    sys.exit(main())
