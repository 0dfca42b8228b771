"""Cost of the token chunking in RowParallelLinear._gemm_ar_overlapped on one MI355X.

At TP > 1 a prefill-sized row-parallel GEMM (o_proj / down_proj) runs as n token chunks so each
chunk's RCCL all-reduce overlaps the next chunk's GEMM (models/layers.py).  Chunking is only a
win if the chunked GEMMs cost less extra time than the all-reduce they hide.  This times, per
rank-local shape (weights [N, K/TP]), the unchunked GEMM against the same chunk loop without
the all-reduce (graph-replayed, hipBLASLt via torch.matmul), and prints the all-reduce payload
per step so the break-even link rate can be read off:  overhead_us = chunked - unchunked; the
overlap pays when the hidden all-reduce time (all but the last chunk's) exceeds it.

usage: python scripts/bench_tp_chunks.py [--m 1024 2048 4096 8192]
"""
import argparse
import json

import torch

# (name, N = hidden, K per rank, TP)
SHAPES = [
    ("70b_tp8_o", 8192, 8192 // 8, 8),
    ("70b_tp8_down", 8192, 28672 // 8, 8),
    ("70b_tp4_down", 8192, 28672 // 4, 4),
    ("8b_tp2_o", 4096, 4096 // 2, 2),
    ("8b_tp2_down", 4096, 14336 // 2, 2),
]


def graph_time(fn, iters=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(iters):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = float("inf")
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1000.0 / iters)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, nargs="*", default=[1024, 2048, 4096, 8192])
    ap.add_argument("--min-tokens", type=int, default=1024)   # EIA_TP_OVERLAP_MIN_TOKENS
    ap.add_argument("--max-chunks", type=int, default=4)      # _OVERLAP_MAX_CHUNKS
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    for name, N, K, tp in SHAPES:
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        for M in a.m:
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            n = max(2, min(a.max_chunks, M // a.min_tokens * 2))
            step = -(-M // n)

            def whole():
                torch.matmul(x, w.t(), out=y)

            def chunked():
                for s in range(0, M, step):
                    e = min(M, s + step)
                    torch.matmul(x[s:e], w.t(), out=y[s:e])

            t1, tn = graph_time(whole), graph_time(chunked)
            ar_mb = M * N * 2 / 1e6
            # the first n-1 chunks' reductions can hide behind later GEMMs
            hidden_mb = ar_mb * (n - 1) / n
            over = tn - t1
            print(json.dumps({
                "shape": name, "M": M, "N": N, "K_rank": K, "tp": tp, "chunks": n,
                "gemm_us": round(t1, 1), "chunked_us": round(tn, 1), "overhead_us": round(over, 1),
                "tflops": round(2 * M * N * K / t1 / 1e6, 1), "ar_payload_mb": round(ar_mb, 2),
                # ring all-reduce moves 2 (tp-1)/tp of the payload per GPU; break-even bus rate
                "breakeven_GBps": (round(2 * (tp - 1) / tp * hidden_mb * 1e3 / over, 1)
                                   if over > 0 else None)}), flush=True)


if __name__ == "__main__":
    main()
