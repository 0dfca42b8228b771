#!/usr/bin/env python3
"""Decode-attention microbenchmark (K1): graph-timed paged_decode for a batch of sequences,
sweeping the partition count P and the in-kernel merge vs the separate reduce kernel.
Reports us/call and effective KV bandwidth."""
import argparse
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from enterprise_inference_amd.ops import attention  # noqa: E402


FLUSH = None


def graph_time(fn, iters=50):
    if FLUSH is not None:       # evict the MALL before every call; the flush alone is subtracted
        inner = fn

        def fn():
            torch.sum(FLUSH[0], 0, out=FLUSH[1])   # read-only sweep: leaves nothing dirty
            inner()
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        with torch.cuda.graph(g, stream=s):
            for _ in range(iters):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(3):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) / iters * 1e3)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, nargs="+", default=[1, 16, 65, 128])
    ap.add_argument("--ctx", type=int, nargs="+", default=[192, 1024, 4096])
    ap.add_argument("--hq", type=int, default=32)
    ap.add_argument("--hkv", type=int, default=8)
    ap.add_argument("--d", type=int, default=128)
    ap.add_argument("--bs", type=int, default=128)
    ap.add_argument("--flush-mb", type=int, default=0,
                    help="copy this many MB before every call (cold Infinity Cache, like the "
                         "engine, where 16 GB of weights stream between two uses of a layer's KV)")
    ap.add_argument("--pool-blocks", type=int, default=0,
                    help="allocate a KV pool of this many blocks and spread the batch's blocks "
                         "over it at random (engine-sized pools)")
    ap.add_argument("--p-only", type=int, nargs="*", default=None, help="partition counts to time")
    ap.add_argument("--fused-sk", type=int, default=0,
                    help="also time the fused RoPE form (eia_paged_decode_rope) fed by sk fp32 "
                         "split-K slabs, as in the engine's pure-decode steps")
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    global FLUSH
    flush_us = 0.0
    if a.flush_mb:
        n = a.flush_mb * (1 << 20) // 4
        FLUSH = (torch.ones(n, device=dev), torch.zeros((), device=dev))
        flush_us = graph_time(lambda: None)
    for B in a.batch:
        for L in a.ctx:
            nbs = math.ceil(L / a.bs)
            nb = max(B * nbs + 1, a.pool_blocks)
            k = torch.empty(nb, a.hkv, a.bs, a.d, device=dev, dtype=bf)
            v = torch.empty(nb, a.hkv, a.d, a.bs, device=dev, dtype=bf)
            bt = torch.randperm(nb - 1, device=dev)[:B * nbs].view(B, nbs).to(torch.int32)
            used = bt.flatten().long()
            k[used] = (torch.randn(used.numel(), a.hkv, a.bs, a.d, device=dev) * 0.5).to(bf)
            v[used] = (torch.randn(used.numel(), a.hkv, a.d, a.bs, device=dev) * 0.5).to(bf)
            sl = torch.full((B,), L, dtype=torch.int32, device=dev)
            q = torch.randn(B, a.hq, a.d, device=dev, dtype=bf)
            out = torch.empty_like(q)
            kv_bytes = B * L * a.hkv * a.d * 2 * 2
            res = []
            for P in (a.p_only or (1, 2, 4, 8)):
                po = torch.empty(B * a.hq * P * a.d, device=dev)
                pml = torch.empty(B * a.hq * P * 2, device=dev)
                for fused in ((False,) if P == 1 else (False, True)):
                    cnt = torch.zeros(B * a.hq, dtype=torch.int32, device=dev) if fused else None
                    t = graph_time(lambda: attention.paged_decode(
                        q, k, v, bt, sl, a.d ** -0.5, P, po, pml, out=out, part_cnt=cnt))
                    res.append((round(t - flush_us, 2), P, fused))
            # graph-style: grid for Pmax=8, P chosen per call on device (model runner path)
            Pm = 8
            po = torch.empty(B * a.hq * Pm * a.d, device=dev)
            pml = torch.empty(B * a.hq * Pm * 2, device=dev)
            pd = torch.tensor([attention.decode_partitions(B, a.hkv, a.hq, L)], dtype=torch.int32,
                              device=dev)
            t = graph_time(lambda: attention.paged_decode(
                q, k, v, bt, sl, a.d ** -0.5, Pm, po, pml, out=out, p_dyn=pd))
            dyn = (round(t - flush_us, 2), int(pd.item()))
            if a.fused_sk:
                from enterprise_inference_amd.ops._dispatch import lib, ptr, stream
                ntot = a.hq + 2 * a.hkv
                part = torch.randn(a.fused_sk, B, ntot * a.d, device=dev) * 0.05
                pos = torch.full((B,), L - 1, dtype=torch.int32, device=dev)
                cs = torch.randn(L + 1, a.d, device=dev)
                slot = (bt[:, (L - 1) // a.bs].long() * a.bs + (L - 1) % a.bs).to(torch.int32)
                for P in (a.p_only or (1, 2)):
                    po = torch.empty(B * a.hq * P * a.d, device=dev)
                    pml = torch.empty(B * a.hq * P * 2, device=dev)
                    cnt = torch.zeros(B * a.hq, dtype=torch.int32, device=dev)

                    def fused_call():
                        rc = lib().eia_paged_decode_rope(
                            None, 0, ptr(part), a.fused_sk, None, None, None, 1e-6, ptr(pos),
                            ptr(cs), ptr(slot), B, ptr(k), ptr(v), ptr(bt), bt.stride(0), ptr(sl),
                            ptr(out), out.stride(0), ptr(po) if P > 1 else None,
                            ptr(pml) if P > 1 else None, ptr(cnt) if P > 1 else None,
                            float(a.d ** -0.5), B, a.hq, a.hkv, a.d, a.bs, P, 0, 0, None,
                            stream(out))
                        assert rc == 0, rc
                    t = graph_time(fused_call)
                    res.append((round(t - flush_us, 2), P, "rope"))
            res.sort(key=lambda r: r[0])
            auto = attention.decode_partitions(B, a.hkv, a.hq, L)
            print(json.dumps({"B": B, "ctx": L, "best_us": res[0][0], "best_P": res[0][1],
                              "fused": res[0][2], "TBps": round(kv_bytes / res[0][0] / 1e6, 2),
                              "heuristic_P": auto, "dyn_us_P": dyn, "all": res,
                              "flush_mb": a.flush_mb, "flush_us": round(flush_us, 2),
                              "pool_blocks": nb}), flush=True)


if __name__ == "__main__":
    main()
