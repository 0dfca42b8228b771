#!/usr/bin/env python3
"""Tune the prefill (large-M) GEMMs with PyTorch TunableOp and ship the winners in-tree.

Prefill GEMMs go through F.linear -> hipBLASLt, whose default heuristic pick ran the 8B
prefill at ~1.5 PFLOP/s (profiles/rocprof_r1_prefill_long.md).  TunableOp times every
hipBLASLt/rocBLAS solution for each exact (M, N, K) and records the fastest; the engine loads
the file at start-up with tuning OFF (enterprise_inference_amd/ops/gemm.py
enable_prefill_tuning), so shapes not in the file keep the default pick and nothing is ever
timed inside a serving step.

    python scripts/tune_prefill_gemm.py --model 8b --out enterprise_inference_amd/ops/tunableop_mi355x.csv
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = {   # (N, K) of the dense projections: QKV, O, gate_up, down, per model
    "8b": [(6144, 4096), (4096, 4096), (28672, 4096), (4096, 14336)],
    "70b": [(10240, 8192), (8192, 8192), (57344, 8192), (8192, 28672)],
}


def timeit(fn, iters=20):
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
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", nargs="*", default=["8b"])
    ap.add_argument("--m", type=int, nargs="*", default=[8192, 4096, 2048, 192])
    ap.add_argument("--out", default="enterprise_inference_amd/ops/tunableop_mi355x.csv")
    ap.add_argument("--persist", action="store_true",
                    help="also copy the results into the PVC tuning cache ($EIA_CACHE_DIR)")
    a = ap.parse_args()
    t = torch.cuda.tunable
    dev, bf = "cuda", torch.bfloat16
    cases = [(m, n, k) for mod in a.model for (n, k) in SHAPES[mod] for m in a.m]
    base = {}
    for m, n, k in cases:
        x = torch.randn(m, k, device=dev, dtype=bf)
        w = torch.randn(n, k, device=dev, dtype=bf)
        base[(m, n, k)] = timeit(lambda: F.linear(x, w))
    t.enable(True)
    t.tuning_enable(True)
    t.set_max_tuning_duration(30)
    t.set_max_tuning_iterations(20)
    t.set_filename(os.path.abspath(a.out))
    t0 = time.time()
    for m, n, k in cases:
        x = torch.randn(m, k, device=dev, dtype=bf)
        w = torch.randn(n, k, device=dev, dtype=bf)
        F.linear(x, w)                       # first call tunes this shape
        torch.cuda.synchronize()
        print(f"tuned {m}x{n}x{k} at {time.time() - t0:.0f}s", flush=True)
    t.tuning_enable(False)
    for m, n, k in cases:
        x = torch.randn(m, k, device=dev, dtype=bf)
        w = torch.randn(n, k, device=dev, dtype=bf)
        us = timeit(lambda: F.linear(x, w))
        fl = 2.0 * m * n * k
        print(json.dumps({"M": m, "N": n, "K": k, "default_us": round(base[(m, n, k)], 1),
                          "tuned_us": round(us, 1),
                          "default_PF": round(fl / base[(m, n, k)] / 1e9, 2),
                          "tuned_PF": round(fl / us / 1e9, 2)}), flush=True)
    # this torch has no tunable.write_file(): write validators + results in TunableOp's CSV form
    with open(a.out, "w") as f:
        for k, v in t.get_validators():
            f.write(f"Validator,{k},{v}\n")
        for op_sig, param_sig, kernel, ms in t.get_results():
            f.write(f"{op_sig},{param_sig},{kernel},{ms}\n")
    t.set_filename(os.path.join("/tmp", "eia_tunableop_exit%d.csv"), True)   # exit write-back
    print("wrote", a.out)
    if a.persist:
        from enterprise_inference_amd.utils.cache_dir import persist
        print("persisted", persist(os.path.abspath(a.out), "tunableop_mi355x.csv"))


if __name__ == "__main__":
    main()
