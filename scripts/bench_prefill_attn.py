#!/usr/bin/env python3
"""Prefill-attention microbenchmark (K2): paged causal prefill of whole prompts, per
tiles-per-wave variant (qt), reporting us/call and causal TFLOP/s.

    python scripts/bench_prefill_attn.py                       # Llama-8B heads, 1x8192, 4x2048, 64x128
    python scripts/bench_prefill_attn.py --shapes 1x8192 --qt 1 2
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from enterprise_inference_amd.ops import attention  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=["1x8192", "4x2048", "65x128"])
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--bs", type=int, default=128)
    ap.add_argument("--qt", type=int, nargs="*", default=None)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--noncausal", action="store_true")
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    qts = a.qt or sorted({1, 2, attention.prefill_tiles(a.d),
                          attention.prefill_variant(a.hq, a.hkv, a.d, a.bs)} |
                         ({attention.PREFILL_LDS | 2} if a.hq % (4 * a.hkv) == 0 else set()))
    for shp in a.shapes:
        B, L = (int(x) for x in shp.split("x"))
        nb = B * ((L + a.bs - 1) // a.bs)
        kc = torch.randn(nb, a.hkv, a.bs, a.d, device=dev, dtype=bf)
        vc = torch.randn(nb, a.hkv, a.d, a.bs, device=dev, dtype=bf)
        bt = torch.randperm(nb, device=dev, dtype=torch.int32).view(B, -1).contiguous()
        sl = torch.full((B,), L, dtype=torch.int32, device=dev)
        cu = torch.arange(0, (B + 1) * L, L, dtype=torch.int32, device=dev)
        q = torch.randn(B * L, a.hq, a.d, device=dev, dtype=bf)
        causal = not a.noncausal
        flops = 4.0 * B * a.hq * a.d * L * ((L + 1) / 2 if causal else L)   # QK^T + PV
        ref = None
        for qt in qts:
            qb = attention.prefill_query_block(a.hq, a.hkv, a.d, qt, block_size=a.bs)
            work = torch.tensor(attention.build_prefill_work([L] * B, qb), dtype=torch.int32,
                                device=dev)
            n = work.numel() // 2

            def fn():
                return attention.paged_prefill(q, kc, vc, bt, sl, cu, work, n, a.d ** -0.5,
                                               causal, qt=qt)
            o = fn()
            torch.cuda.synchronize()
            if ref is None:
                ref = o
            err = (o.float() - ref.float()).abs().max().item()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            print(json.dumps({"shape": shp, "causal": causal, "hq": a.hq, "hkv": a.hkv, "d": a.d, "qt": qt,
                              "us": round(us, 1), "tflops": round(flops / us / 1e6, 1),
                              "max_diff_vs_qt%d" % qts[0]: err}), flush=True)


if __name__ == "__main__":
    main()
