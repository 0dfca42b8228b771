#!/usr/bin/env python3
"""Prompt-sized GEMMs: the K7 MFMA kernel (csrc/kernels/gemm_prefill.hip) against hipBLASLt.

SwiGLU shapes time ours (GEMM + epilogue) against F.linear + act_and_mul (what the prefill
path runs otherwise); plain shapes against F.linear alone.  One JSON line per shape with us
and TFLOP/s (2 M N K flops), and the max |diff| between the two outputs."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

SHAPES = {  # name: (N rows of W, K, swiglu)
    "gate_up_8b": (28672, 4096, True), "down_8b": (4096, 14336, False),
    "qkv_8b": (6144, 4096, False), "gate_up_70b": (57344, 8192, True),
    "gate_up_70b_tp4": (14336, 8192, True), "sq_8k": (8192, 8192, False),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", nargs="*", default=["gate_up_8b", "down_8b", "qkv_8b"])
    ap.add_argument("--m", type=int, nargs="*", default=[8192])
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    import torch
    from enterprise_inference_amd.ops import activation, gemm
    gemm.enable_prefill_tuning()

    def timed(fn):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) * 1e3 / a.iters

    for name in a.shapes:
        N, K, sw = SHAPES[name]
        w = (torch.randn(N, K, device="cuda") * K ** -0.5).to(torch.bfloat16)
        for M in a.m:
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            if sw:
                base = lambda: activation.act_and_mul(torch.nn.functional.linear(x, w), "silu")
            else:
                base = lambda: torch.nn.functional.linear(x, w)
            ours = lambda: gemm.prefill_gemm(x, w, swiglu=sw)
            d = (ours().float() - base().float()).abs().max().item()
            tb, to = timed(base), timed(ours)
            fl = 2.0 * M * N * K
            print(json.dumps({"shape": name, "M": M, "N": N, "K": K, "swiglu": sw,
                              "ours_us": round(to, 1), "ours_TFLOPs": round(fl / to / 1e6, 1),
                              "hipblaslt_us": round(tb, 1), "hipblaslt_TFLOPs": round(fl / tb / 1e6, 1),
                              "speedup": round(tb / to, 3), "max_diff": round(d, 4)}), flush=True)
            del x
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
