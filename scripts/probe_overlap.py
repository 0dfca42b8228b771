#!/usr/bin/env python3
"""Probe which command in an overlapped decode step delays the previous step's event.

Each 'step' = [small pinned H2D copy] -> [graph replay or eager kernels] -> [D2H copy of
64 ints to pinned memory] -> event.  The host launches step k+1 before waiting on step k's
event (the engine's overlapped scheduling) and spends ~0.5 ms of 'host work' per step.  If
the overlap works, the period equals the GPU step time."""
import itertools
import time

import torch


def main():
    dev = "cuda"
    x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    w = [torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16) for _ in range(4)]
    hdr_h = [torch.zeros(4096, dtype=torch.int32, pin_memory=True) for _ in range(2)]
    hdr_d = torch.zeros(4096, dtype=torch.int32, device=dev)
    tok_d = torch.zeros(64, dtype=torch.int32, device=dev)
    tok_h = [torch.zeros(64, dtype=torch.int32, pin_memory=True) for _ in range(2)]

    def body():
        y = x
        for i in range(24):
            y = torch.mm(y, w[i % 4])
        tok_d.copy_(y[0, :64].float().to(torch.int32))
        return y

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
        with torch.cuda.graph(g, stream=s):
            body()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    gstep = (time.perf_counter() - t0) / 20
    print(f"graph step alone: {gstep * 1e3:.3f} ms", flush=True)
    for h2d, graph, d2h in itertools.product((True, False), (True, False), (True, False)):
        torch.cuda.synchronize()
        prev = None
        n = 40
        waits = 0.0
        t0 = time.perf_counter()
        for k in range(n):
            p = k & 1
            if h2d:
                hdr_h[p][:8] = k
                hdr_d.copy_(hdr_h[p], non_blocking=True)
            if graph:
                g.replay()
            else:
                body()
            if d2h:
                tok_h[p].copy_(tok_d, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
            if prev is not None:
                tw = time.perf_counter()
                prev.synchronize()
                waits += time.perf_counter() - tw
            t = time.perf_counter()
            while time.perf_counter() - t < 0.0005:     # host work of a step
                pass
            prev = ev
        prev.synchronize()
        per = (time.perf_counter() - t0) / n
        print(f"h2d={h2d:d} graph={graph:d} d2h={d2h:d}: {per * 1e3:.3f} ms/step "
              f"(+{(per - gstep) * 1e3:.3f} over GPU), wait {waits / n * 1e3:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
