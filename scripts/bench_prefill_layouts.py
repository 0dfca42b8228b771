#!/usr/bin/env python3
"""Prefill GEMM: which weight layout lets the library reach the most MFMA throughput.

For the 8B (and optionally 70B) prefill shapes at M tokens, times the library GEMM for
  tn : y = x @ W^T, W [N, K] row-major (what F.linear runs today)
  nn : y = x @ Wt,  Wt [K, N] row-major (a transposed weight copy)
each with TunableOp tuning ON (the best hipBLASLt / rocBLAS solution for that layout) and
with the default heuristic pick, and prints TFLOP/s.  Cold-ish: a 512 MB sweep between reps
would dominate at these sizes, so reps are back to back (the weights do not fit the
Infinity Cache anyway: 235 MB gate_up).

  python scripts/bench_prefill_layouts.py --m 8192 --out gpurun_out/prefill_layouts.md
"""
from __future__ import annotations

import argparse
import os
import statistics
import sys
import tempfile

SHAPES = {
    "8b": [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672, 4096), ("down", 4096, 14336)],
    "70b": [("qkv", 10240, 8192), ("o", 8192, 8192), ("gate_up", 57344, 8192), ("down", 8192, 28672)],
}


def timeit(fn, reps: int = 20) -> float:
    import torch
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return statistics.median(ts)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="+", default=[8192])
    ap.add_argument("--models", nargs="+", default=["8b"])
    ap.add_argument("--tune", action="store_true", help="TunableOp tuning on (slow)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    if a.tune:
        t = torch.cuda.tunable
        t.enable(True)
        t.tuning_enable(True)
        t.set_max_tuning_duration(30)
        t.set_max_tuning_iterations(20)
        t.set_filename(os.path.join(tempfile.gettempdir(), "eia_layout_tune%d.csv"), True)
    dev = "cuda"
    lines = [f"# Prefill GEMM layouts ({'TunableOp tuned' if a.tune else 'default pick'})", "",
             "| model | gemm | M | N | K | tn ms | tn TFLOP/s | nn ms | nn TFLOP/s |",
             "|---|---|---:|---:|---:|---:|---:|---:|---:|"]
    for model in a.models:
        for name, N, K in SHAPES[model]:
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            wt = w.t().contiguous()
            for M in a.m:
                x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
                y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                t_tn = timeit(lambda: torch.matmul(x, w.t(), out=y))
                ref = y.clone()
                t_nn = timeit(lambda: torch.matmul(x, wt, out=y))
                err = (y.float() - ref.float()).abs().max().item()
                fl = 2.0 * M * N * K
                lines.append(f"| {model} | {name} | {M} | {N} | {K} | {t_tn:.3f} | {fl / t_tn / 1e9:.0f} | "
                             f"{t_nn:.3f} | {fl / t_nn / 1e9:.0f} |")
                print(lines[-1], "max|tn-nn|", err, flush=True)
                del x, y, ref
            del w, wt
            torch.cuda.empty_cache()
    text = "\n".join(lines) + "\n"
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text)
    return 0


if __name__ == "__main__":
    sys.exit(main())
