#!/usr/bin/env python3
"""Prefill GEMM at ragged M: hipBLASLt's default pick vs a 256-row-aligned body + remainder.

The TunableOp sweep (profiles/tune_prefill_gemm_r1.log) showed M = 8320 running up to 1.7x
slower than M = 8192 on the same (N, K).  Prefill M is the step's token count, i.e. arbitrary,
so this measures, per (M, N, K): F.linear on all rows; the aligned body (M - M % 256 rows,
a contiguous view, written in place through matmul(out=)) plus the remainder rows through
ops.gemm.linear (skinny kernel when <= 128 rows); and zero-padding M up to a multiple of 256.

    python scripts/probe_prefill_split.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from enterprise_inference_amd.ops import gemm  # noqa: E402

SHAPES = [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)]
MS = [320, 600, 1100, 2100, 3000, 4100, 5000, 6200, 7000, 8100, 8320]


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def main():
    dev, bf = "cuda", torch.bfloat16
    for n, k in SHAPES:
        w = torch.randn(n, k, device=dev, dtype=bf) * 0.02
        for m in MS:
            x = torch.randn(m, k, device=dev, dtype=bf)
            out = torch.empty(m, n, device=dev, dtype=bf)
            body = m - m % 256
            rem = m - body

            def split():
                torch.matmul(x[:body], w.t(), out=out[:body])
                if rem:
                    out[body:] = gemm.linear(x[body:], w)

            mp = body + (256 if rem else 0)
            xp = torch.zeros(mp, k, device=dev, dtype=bf)

            def pad():
                xp[:m].copy_(x)
                return F.linear(xp, w)

            t_full = timeit(lambda: F.linear(x, w))
            t_split = timeit(split) if body else None
            t_pad = timeit(pad)
            ref = F.linear(x, w).float()
            split()
            err = (out.float() - ref).abs().max().item()
            print(json.dumps({"M": m, "N": n, "K": k, "full_us": round(t_full, 1),
                              "split_us": t_split and round(t_split, 1),
                              "pad_us": round(t_pad, 1), "split_err": err}), flush=True)
            del x, out, xp
        del w
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
