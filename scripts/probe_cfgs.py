#!/usr/bin/env python3
"""Time chosen skinny-GEMM cfgs over split-K values on the decode shapes (cold weights).
Usage: probe_cfgs.py [--m 65] [--cfgs 19 3 146 ...] [--shapes qkv_8b ...]"""
import argparse
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from enterprise_inference_amd.ops import gemm  # noqa: E402
from scripts.bench_gemm import SHAPES, graph_time  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=65)
    ap.add_argument("--cfgs", type=int, nargs="+", default=[3, 19] + list(gemm.GLDS_CFGS))
    ap.add_argument("--shapes", nargs="+", default=["qkv_8b", "o_8b", "gate_up_8b", "down_8b"])
    ap.add_argument("--sks", type=int, nargs="+", default=[1, 2, 4, 8])
    a = ap.parse_args()
    M = a.m
    for name in a.shapes:
        N, K, swiglu = SHAPES[name]
        wb = N * K * 2
        pool = max(2, int(600e6 // wb) + 1)
        ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(pool)]
        x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
        for cfg in a.cfgs:
            row = []
            for sk in ([1] if swiglu else a.sks):
                if not gemm.valid(N, K, swiglu, cfg, sk, M=M):
                    continue
                if swiglu:
                    f = lambda i, cfg=cfg: gemm.swiglu_gemm(x, ws[i % pool], cfg=cfg)
                else:
                    f = lambda i, cfg=cfg, sk=sk: gemm.skinny(x, ws[i % pool], cfg=cfg, sk=sk,
                                                               defer_reduce=True)
                t = graph_time(f, 20)
                row.append(f"sk{sk} {t:6.2f}us {wb / t / 1e6:4.2f}TB/s")
            print(f"{name:12s} cfg {cfg:3d}: " + " | ".join(row), flush=True)
        del ws
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
