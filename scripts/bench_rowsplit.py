#!/usr/bin/env python3
"""Decode GEMMs just past the skinny kernel's 128 rows: hipBLASLt vs the skinny kernel on row
halves.

Batches of 129-256 rows (decode at 135-210 users -- the suggest / describe sizing rows -- and
the mixed steps that add a short prompt to a full decode batch) leave the skinny kernel
(MAX_M 128) for hipBLASLt, whose picks at these M stream the weight at 1-3 TB/s.  This times,
per 8B shape and M, with a 512 MB sweep before every rep (the engine streams ~435 MB of other
weights between two uses of a layer's):
  lib    : F.linear (+ act_and_mul for gate_up)
  split2 : two skinny launches over row halves (SwiGLU fused for gate_up); the second half
           re-reads a weight the first just streamed
and prints us (graph replay, as in the engine) and the weight-stream rate.

  python scripts/bench_rowsplit.py --m 136 192 256 --out gpurun_out/rowsplit.md
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SHAPES = {"8b": [("qkv", 6144, 4096, False), ("o", 4096, 4096, False),
                 ("gate_up", 28672, 4096, True), ("down", 4096, 14336, False)],
          "70b-tp8": [("qkv", 1280, 8192, False), ("o", 8192, 1024, False),
                      ("gate_up", 7168, 8192, True), ("down", 8192, 3584, False)]}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[136, 160, 192, 224, 256])
    ap.add_argument("--models", nargs="+", default=["8b"])
    ap.add_argument("--reps", type=int, default=15)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    import torch.nn.functional as F

    from enterprise_inference_amd.ops import activation, gemm

    gemm.enable_prefill_tuning()
    flush = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")

    def timed(fn):
        # replayed from a HIP graph, as the engine's decode steps are: the eager host cost of
        # the split form's extra launches would otherwise be what is measured
        fn()
        torch.cuda.synchronize()
        st = torch.cuda.Stream()
        st.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(st):
            fn()
            with torch.cuda.graph(g, stream=st):
                fn()
        torch.cuda.current_stream().wait_stream(st)
        torch.cuda.synchronize()
        ts = []
        for i in range(a.reps + 2):
            flush.add_(1)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            if i >= 2:
                ts.append(1e3 * s.elapsed_time(e))
        return statistics.median(ts)

    lines = ["| model | gemm | M | lib us | split2 us | lib TB/s | split2 TB/s | max abs diff |",
             "|---|---|---:|---:|---:|---:|---:|---:|"]
    for model in a.models:
        for name, N, K, sw in SHAPES[model]:
            w = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02
            for M in a.m:
                x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
                h = (M + 1) // 2
                if sw:
                    def lib_fn():
                        return activation.act_and_mul(F.linear(x, w), "silu")

                    def split_fn():
                        return torch.cat([gemm.swiglu_gemm(x[:h], w), gemm.swiglu_gemm(x[h:], w)])
                else:
                    def lib_fn():
                        return F.linear(x, w)

                    def split_fn():
                        return torch.cat([gemm.skinny(x[:h], w), gemm.skinny(x[h:], w)])
                ok = gemm.skinny_ok(x[:h], w, swiglu=sw) and gemm.skinny_ok(x[h:], w, swiglu=sw)
                if not ok:
                    lines.append(f"| {model} | {name} | {M} | - | not skinny | | | |")
                    continue
                d = (lib_fn().float() - split_fn().float()).abs().max().item()
                t_lib, t_split = timed(lib_fn), timed(split_fn)
                gb = N * K * 2 / 1e9
                lines.append(f"| {model} | {name} | {M} | {t_lib:.1f} | {t_split:.1f} | "
                             f"{gb / t_lib * 1e3:.2f} | {gb / t_split * 1e3:.2f} | {d:.3g} |")
                print(lines[-1], flush=True)
            del w
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
