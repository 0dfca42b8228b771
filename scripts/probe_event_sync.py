#!/usr/bin/env python3
"""Probe: does waiting on an event recorded after step A also wait for work enqueued
after it (step B)?  Overlapped scheduling relies on it NOT doing so."""
import time

import torch


def busy(x, n):
    for _ in range(n):
        x = x @ x
        x = x / x.norm()
    return x


def main():
    x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
    busy(x, 4)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    busy(x, 40)
    torch.cuda.synchronize()
    t_a = time.perf_counter() - t0
    host = torch.zeros(64, dtype=torch.int32, pin_memory=True)
    dev = torch.arange(64, dtype=torch.int32, device="cuda")
    for mode in ("event", "event_blocking", "query_poll", "side_stream"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        busy(x, 40)                                   # step A
        if mode == "side_stream":
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                host.copy_(dev, non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(s)
        else:
            host.copy_(dev, non_blocking=True)
            ev = torch.cuda.Event(blocking=(mode == "event_blocking"))
            ev.record()
        t_enq_a = time.perf_counter() - t0
        busy(x, 40)                                   # step B, enqueued before the wait
        t_enq_b = time.perf_counter() - t0
        if mode == "query_poll":
            while not ev.query():
                time.sleep(20e-6)
        else:
            ev.synchronize()
        t_wait = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        print(f"{mode:15s} step={t_a * 1e3:.2f}ms enqA={t_enq_a * 1e3:.2f} enqB={t_enq_b * 1e3:.2f} "
              f"wait_done_at={t_wait * 1e3:.2f} all_done_at={t_all * 1e3:.2f}", flush=True)


if __name__ == "__main__":
    main()
