#!/usr/bin/env python3
"""Per-wave phase timeline of the fused decode attention (diagnostic build).

Loads ``enterprise_inference_amd/_lib/libeia_attn_trace.so`` -- attention.hip built with
-DEIA_ATTN_TRACE (``python scripts/attn_trace.py --build`` on the build host) -- runs ONE
eia_paged_decode_rope call after a 512 MB read sweep (cold Infinity Cache, as in the engine)
and prints, per trace slot, when the waves reach it (us after the first wave started) and the
per-wave phase durations:
  0 entry, 6 entry loads (L, P, position, slot) arrived, 1 prologue entered (the first unit's
  K/V loads issued), 2 prologue done (barrier), 3 unit loop done, 4 cross-wave merge barrier
  passed, 5 output written."""
import argparse
import ctypes
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SO = os.path.join(ROOT, "enterprise_inference_amd", "_lib", "libeia_attn_trace.so")


def build():
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    import build as b
    subprocess.run([b.HIPCC, *b.HIP_FLAGS, "-shared", "-DEIA_ATTN_TRACE",
                    os.path.join(ROOT, "csrc", "kernels", "attention.hip"), "-o", SO], check=True)
    print("built", SO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--batch", type=int, default=65)
    ap.add_argument("--ctx", type=int, default=192)
    ap.add_argument("--sk", type=int, default=4)
    ap.add_argument("--flush-mb", type=int, default=512)
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch
    from enterprise_inference_amd import _native
    lib = ctypes.CDLL(SO)
    P_, I_, L_, F_ = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float
    lib.eia_paged_decode_rope.argtypes = [P_, L_, P_, I_, P_, P_, P_, F_, P_, P_, P_, I_, P_, P_,
                                          P_, I_, P_, P_, L_, P_, P_, P_, F_, I_, I_, I_, I_, I_,
                                          I_, I_, I_, P_, P_, P_]
    lib.eia_attn_set_trace.argtypes = [P_]
    del _native
    dev, bf = "cuda", torch.bfloat16
    B, L, hq, hkv, d, bs = a.batch, a.ctx, 32, 8, 128, 128
    nbs = (L + bs - 1) // bs
    nb = 16384
    k = torch.empty(nb, hkv, bs, d, device=dev, dtype=bf)
    v = torch.empty(nb, hkv, d, bs, device=dev, dtype=bf)
    bt = torch.randperm(nb - 1, device=dev)[:B * nbs].view(B, nbs).to(torch.int32)
    used = bt.flatten().long()
    k[used] = (torch.randn(used.numel(), hkv, bs, d, device=dev) * 0.5).to(bf)
    v[used] = (torch.randn(used.numel(), hkv, d, bs, device=dev) * 0.5).to(bf)
    sl = torch.full((B,), L, dtype=torch.int32, device=dev)
    ntot = hq + 2 * hkv
    part = torch.randn(a.sk, B, ntot * d, device=dev) * 0.05
    pos = torch.full((B,), L - 1, dtype=torch.int32, device=dev)
    cs = torch.randn(L + 1, d, device=dev)
    slot = (bt[:, (L - 1) // bs].long() * bs + (L - 1) % bs).to(torch.int32)
    out = torch.empty(B, hq, d, device=dev, dtype=bf)
    trace = torch.zeros(B * hkv * 32, dtype=torch.int64, device=dev)
    assert lib.eia_attn_set_trace(ctypes.c_void_p(trace.data_ptr())) == 0
    flush = torch.ones(a.flush_mb * (1 << 18), device=dev)
    acc = torch.zeros((), device=dev)
    st = torch.cuda.current_stream().cuda_stream

    def call():
        rc = lib.eia_paged_decode_rope(None, 0, part.data_ptr(), a.sk, None, None, None, 1e-6,
                                       pos.data_ptr(), cs.data_ptr(), slot.data_ptr(), B,
                                       k.data_ptr(), v.data_ptr(), bt.data_ptr(), bt.stride(0),
                                       sl.data_ptr(), out.data_ptr(), out.stride(0), None, None,
                                       None, d ** -0.5, B, hq, hkv, d, bs, 1, 0, 0, None, None, st)
        assert rc == 0, rc
    for _ in range(3):
        torch.sum(flush, 0, out=acc)
        trace.zero_()
        call()
    torch.cuda.synchronize()
    t = trace.view(B * hkv, 4, 8).cpu().double() / 100.0   # 100 MHz ticks -> us
    t0 = t[:, :, 0][t[:, :, 0] > 0].min()
    names = ["entry", "prologue in", "prologue out", "units done", "merge barrier", "stored",
             "L arrived", "-"]
    print(f"B {B} ctx {L} sk {a.sk}: {B * hkv} workgroups x 4 waves, cold ({a.flush_mb} MB sweep)")
    for sl_ in range(8):
        x = t[:, :, sl_].flatten()
        x = x[x > 0] - t0
        if x.numel():
            q = torch.quantile(x, torch.tensor([0.0, 0.5, 0.9, 1.0], dtype=torch.float64))
            print(f"  slot {sl_} {names[sl_]:>14}: min {q[0]:6.2f}  p50 {q[1]:6.2f}  p90 {q[2]:6.2f}"
                  f"  max {q[3]:6.2f} us")
    for a_, b_ in ((0, 6), (6, 1), (1, 2), (2, 3), (3, 4), (4, 5), (0, 5)):
        ok = (t[:, :, a_] > 0) & (t[:, :, b_] > 0)
        dlt = (t[:, :, b_] - t[:, :, a_])[ok]
        if dlt.numel():
            q = torch.quantile(dlt, torch.tensor([0.5, 0.9, 1.0], dtype=torch.float64))
            print(f"  {names[a_]:>14} -> {names[b_]:<14}: p50 {q[0]:6.2f}  p90 {q[1]:6.2f}"
                  f"  max {q[2]:6.2f} us")


if __name__ == "__main__":
    main()
