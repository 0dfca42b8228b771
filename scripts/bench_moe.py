#!/usr/bin/env python3
"""MoE layer microbenchmark (K9): fused_moe at Mixtral-8x7B shapes (E 8, top-2, H 4096,
I 14336) for decode- and prefill-sized token counts, grouped kernels vs the per-expert
hipBLASLt GEMMs on the sorted rows (one offsets read-back); reports us/call and the expert-GEMM TFLOP/s.

    python scripts/bench_moe.py --tokens 65 2048 8192
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from enterprise_inference_amd.ops import moe  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, nargs="*", default=[65, 2048, 8192])
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--topk", type=int, default=2)
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--inter", type=int, default=14336)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    E, k, H, I = a.experts, a.topk, a.hidden, a.inter
    w13 = (torch.randn(E, 2 * I, H, device=dev) * H ** -0.5).to(bf)
    w2 = (torch.randn(E, H, I, device=dev) * I ** -0.5).to(bf)
    for T in a.tokens:
        x = torch.randn(T, H, device=dev, dtype=bf)
        w, ids = moe.topk_route(torch.randn(T, E, device=dev), k, True)
        flops = 2.0 * T * k * (2 * I * H + H * I)
        res = {}
        for name, fn in (("grouped", lambda: moe._fused_moe_grouped(x, w13, w2, w, ids, 0, E,
                                                                    mfma=T * k / E > 96)),
                         ("per_expert", lambda: moe._fused_moe_sorted_blas(x, w13, w2, w, ids, 0,
                                                                           E, "silu"))):
            out = fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) / a.iters * 1e3
            res[name] = (us, out)
        diff = (res["grouped"][1].float() - res["per_expert"][1].float()).abs().max().item()
        print(json.dumps({"tokens": T, "E": E, "k": k, "H": H, "I": I,
                          "grouped_us": round(res["grouped"][0], 1),
                          "grouped_tflops": round(flops / res["grouped"][0] / 1e6, 1),
                          "per_expert_us": round(res["per_expert"][0], 1),
                          "per_expert_tflops": round(flops / res["per_expert"][0] / 1e6, 1),
                          "max_diff": diff}), flush=True)


if __name__ == "__main__":
    main()
