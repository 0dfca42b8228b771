#!/usr/bin/env python3
"""Decode MLP half of a Llama layer, one launch vs two (csrc/kernels/mlp_fused.hip):

  two   : SwiGLU skinny GEMM (gate_up, tuned cfg) + split-K down skinny GEMM (tuned cfg)
  fused : eia_mlp_fused (balanced producers -> split-K down consumers, one launch)
  prod  : fused, producers only (the gate_up half)
  R<n>  : fused with n rows of gate / up per producer (R<n>prod: producers only)

Weights rotate over --copies sets (> the 256 MB Infinity Cache), so every call streams from
HBM as in the engine.  --trace prints the fused launch's per-workgroup timeline (100 MHz wall
clock): producer stream end / exit, consumer weights-issued / wait-passed / exit.
"""
import argparse
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="*", default=[65])
    ap.add_argument("--shape", default="8b", choices=["8b", "70b"])
    ap.add_argument("--copies", type=int, default=4)
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--trace", action="store_true")
    ap.add_argument("--rows", type=int, nargs="*", default=[], help="extra producer row counts R")
    a = ap.parse_args()
    import torch
    from enterprise_inference_amd.ops import gemm
    from enterprise_inference_amd.ops._dispatch import lib, ptr, stream
    H, I = (4096, 14336) if a.shape == "8b" else (8192, 28672)
    dev, bf = "cuda", torch.bfloat16
    wgu = [(torch.randn(2 * I, H, device=dev) * H ** -0.5).to(bf) for _ in range(a.copies)]
    wd = [(torch.randn(H, I, device=dev) * I ** -0.5).to(bf) for _ in range(a.copies)]
    L = lib()
    for M in a.m:
        x = torch.randn(M, H, device=dev, dtype=bf)
        sk = gemm.mlp_fused_split(M, H, I)
        h = torch.empty(M, I, device=dev, dtype=bf)
        part = torch.empty(sk, M, H, device=dev, dtype=torch.float32)
        sync = gemm.mlp_sync_buffer(x.device)
        tr = torch.zeros(4 * 1024, dtype=torch.int64, device=dev)

        def fused(i, flags=0, trace=None):
            gemm.check(L.eia_mlp_fused_dbg(ptr(x), x.stride(0), ptr(wgu[i]), ptr(wd[i]), ptr(h),
                                           ptr(part), ptr(sync), M, H, I, sk, flags,
                                           ptr(trace), stream(x)), "mlp_fused_dbg")

        def two(i):
            hh = gemm.swiglu_gemm(x, wgu[i])
            gemm.skinny(hh, wd[i], defer_reduce=True)

        variants = {"two": two, "fused": fused, "prod": lambda i: fused(i, 1)}
        for R in a.rows:
            variants[f"R{R}"] = lambda i, R=R: fused(i, R << 8)
            variants[f"R{R}prod"] = lambda i, R=R: fused(i, (R << 8) | 1)
        res = {k: [] for k in variants}
        for it in range(a.iters):
            for name, fn in variants.items():
                i = it % a.copies
                e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                e0.record()
                fn(i)
                e1.record()
                e1.synchronize()
                if it >= 3:
                    res[name].append(e0.elapsed_time(e1) * 1e3)
        mb = (2 * I * H + H * I) * 2 / 1e6
        print(f"M={M:3d} sk={sk} {mb:.0f}MB", flush=True)
        for k, v in res.items():
            print(f"  {k:10s} p50 {statistics.median(v):7.2f} us  min {min(v):7.2f} us", flush=True)
        if a.trace:
            import ctypes
            rr = ctypes.c_int(int(os.environ.get("EIA_MLP_ROWS", "0")))
            L.eia_mlp_fused_plan(M, H, I, sk, ctypes.byref(rr))
            P = I // rr.value
            print(f"  R={rr.value} producers={P} consumers={(H // 128) * sk}")
            C = (H // 128) * sk
            for _ in range(3):
                fused(1 % a.copies)
            torch.cuda.synchronize()
            fused(0, 0, tr)
            torch.cuda.synchronize()
            t = tr[:4 * (P + C)].view(-1, 4).cpu().double()
            t0 = t[:, 0].min()
            t = (t - t0) / 100.0        # 100 MHz -> us
            pr, co = t[:P], t[P:P + C]

            def q(v):
                v = sorted(v.tolist())
                return f"min {v[0]:6.2f} p50 {v[len(v) // 2]:6.2f} p90 {v[int(len(v) * .9)]:6.2f} max {v[-1]:6.2f}"
            print("  producer entry      ", q(pr[:, 0]))
            print("  producer X staged   ", q(pr[:, 1]))
            print("  producer stream done", q(pr[:, 2]))
            print("  producer exit       ", q(pr[:, 3]))
            print("  consumer entry      ", q(co[:, 0]))
            print("  consumer W issued   ", q(co[:, 1]))
            print("  consumer wait passed", q(co[:, 2]))
            print("  consumer exit       ", q(co[:, 3]))
            print("  consumer stream     ", q(co[:, 3] - co[:, 2]))
            print("  producer stream     ", q(pr[:, 2] - pr[:, 0]))


if __name__ == "__main__":
    main()
