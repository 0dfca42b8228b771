#!/usr/bin/env python3
"""Probe the fixed cost of one skinny-GEMM launch inside a graph: time vs K at fixed N
(weights from a pool larger than the Infinity Cache, and one hot weight), plus an empty
kernel.  t(K) = floor + bytes / bandwidth; the floor is what kernel fusion could recover."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from enterprise_inference_amd.ops import gemm  # noqa: E402
from scripts.bench_gemm import graph_time  # noqa: E402


def main():
    M = int(os.environ.get("GEMM_M", "65"))
    z = torch.zeros(64, device="cuda")
    print(f"empty add_ kernel: {graph_time(lambda i: z.add_(1.0), 50):.2f} us", flush=True)
    for N, cfg in ((6144, 19), (4096, 17), (28672, 3)):
        for K in (128, 512, 1024, 2048, 4096):
            x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
            wb = N * K * 2
            pool = max(2, int(600e6 // wb) + 1)
            ws = [(torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16) for _ in range(pool)]
            for sk in (1, 2, 4):
                if not gemm.valid(N, K, False, cfg, sk, M=M):
                    continue
                tc = graph_time(lambda i: gemm.skinny(x, ws[i % pool], cfg=cfg, sk=sk, defer_reduce=True), 40)
                th = graph_time(lambda i: gemm.skinny(x, ws[0], cfg=cfg, sk=sk, defer_reduce=True), 40)
                print(f"N={N} K={K} cfg={cfg} sk={sk} MB={wb / 1e6:.1f} cold {tc:.2f} us "
                      f"({wb / tc / 1e6:.2f} TB/s)  hot {th:.2f} us", flush=True)
            del ws
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
