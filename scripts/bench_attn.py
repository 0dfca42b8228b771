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


def graph_time(fn, iters=50):
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
    a = ap.parse_args()
    dev, bf = "cuda", torch.bfloat16
    for B in a.batch:
        for L in a.ctx:
            nbs = math.ceil(L / a.bs)
            nb = B * nbs + 1
            k = (torch.randn(nb, a.hkv, a.bs, a.d, device=dev) * 0.5).to(bf)
            v = (torch.randn(nb, a.hkv, a.d, a.bs, device=dev) * 0.5).to(bf)
            bt = torch.randperm(nb - 1, device=dev)[:B * nbs].view(B, nbs).to(torch.int32)
            sl = torch.full((B,), L, dtype=torch.int32, device=dev)
            q = torch.randn(B, a.hq, a.d, device=dev, dtype=bf)
            out = torch.empty_like(q)
            kv_bytes = B * L * a.hkv * a.d * 2 * 2
            res = []
            for P in (1, 2, 4, 8):
                po = torch.empty(B * a.hq * P * a.d, device=dev)
                pml = torch.empty(B * a.hq * P * 2, device=dev)
                for fused in ((False,) if P == 1 else (False, True)):
                    cnt = torch.zeros(B * a.hq, dtype=torch.int32, device=dev) if fused else None
                    t = graph_time(lambda: attention.paged_decode(
                        q, k, v, bt, sl, a.d ** -0.5, P, po, pml, out=out, part_cnt=cnt))
                    res.append((round(t, 2), P, fused))
            # graph-style: grid for Pmax=8, P chosen per call on device (model runner path)
            Pm = 8
            po = torch.empty(B * a.hq * Pm * a.d, device=dev)
            pml = torch.empty(B * a.hq * Pm * 2, device=dev)
            pd = torch.tensor([attention.decode_partitions(B, a.hkv, a.hq, L)], dtype=torch.int32,
                              device=dev)
            t = graph_time(lambda: attention.paged_decode(
                q, k, v, bt, sl, a.d ** -0.5, Pm, po, pml, out=out, p_dyn=pd))
            dyn = (round(t, 2), int(pd.item()))
            res.sort()
            auto = attention.decode_partitions(B, a.hkv, a.hq, L)
            print(json.dumps({"B": B, "ctx": L, "best_us": res[0][0], "best_P": res[0][1],
                              "fused": res[0][2], "TBps": round(kv_bytes / res[0][0] / 1e6, 2),
                              "heuristic_P": auto, "dyn_us_P": dyn, "all": res}), flush=True)


if __name__ == "__main__":
    main()
