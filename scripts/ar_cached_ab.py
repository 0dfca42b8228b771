#!/usr/bin/env python3
"""Custom all-reduce (K12) data buffers: uncached (hipDeviceMallocUncached, the default) vs
cached (hipMalloc, EIA_AR_CACHED_DATA=1), timed in the one-GPU W-streams harness (every
'rank' a stream of this process, each on its own hardware queue -- run with
GPU_MAX_HW_QUEUES=8).  Checks every result against the fp32 sum; prints us per call (all W
streams done) per message size, one-shot and two-shot.  What it cannot show: xGMI reads of a
peer's cached buffer (only an 8-GPU run can)."""
import ctypes
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from enterprise_inference_amd import _native
    lib = _native.kernels()
    world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    max_bytes, nblocks = 8 << 20, 16
    for cached in (False, True, False, True):
        own = []

        def alloc(nb, c):
            p = ctypes.c_void_p()
            fn = lib.eia_ar_alloc_cached if c else lib.eia_ar_alloc
            assert fn(ctypes.byref(p), ctypes.c_long(nb)) == 0
            own.append(p.value)
            return p.value
        sigs = [alloc(lib.eia_ar_signal_bytes(), False) for _ in range(world)]
        datas = [alloc(2 * max_bytes, cached) for _ in range(world)]
        sig_arr = (ctypes.c_void_p * world)(*sigs)
        data_arr = (ctypes.c_void_p * world)(*datas)
        streams = [torch.cuda.Stream() for _ in range(world)]
        line = []
        bad = 0
        for n in (8192, 65536, 262144, 1 << 20, 4 << 20):
            elems = n // 2
            for kind in (0, 1):
                base = torch.randn(world, elems, device="cuda").to(torch.bfloat16)
                ts = []
                for it in range(12):
                    xs = [base[r].clone() for r in range(world)]
                    torch.cuda.synchronize()
                    e0 = torch.cuda.Event(enable_timing=True)
                    e1 = [torch.cuda.Event(enable_timing=True) for _ in range(world)]
                    e0.record()
                    for r in range(world):
                        streams[r].wait_event(e0)
                        assert lib.eia_ar_run(ctypes.cast(sig_arr, ctypes.c_void_p),
                                              ctypes.cast(data_arr, ctypes.c_void_p), r, world,
                                              xs[r].data_ptr(), xs[r].data_ptr(), elems,
                                              max_bytes, kind, nblocks,
                                              streams[r].cuda_stream) == 0
                        e1[r].record(streams[r])
                    torch.cuda.synchronize()
                    if it >= 2:
                        ts.append(max(e0.elapsed_time(e) for e in e1) * 1e3)
                    ref = base.float().sum(0)
                    bad += sum(int((xs[r].float() - ref).abs().max().item() > 0.06 * world)
                               for r in range(world))
                line.append(f"{n >> 10}K/{'2s' if kind else '1s'} {statistics.median(ts):.1f}")
                print(f"  W={world} cached={int(cached)} {line[-1]}", flush=True)
        errs = []
        for sp in sigs:
            v = ctypes.c_int(0)
            assert lib.eia_ar_read_err(ctypes.c_void_p(sp), ctypes.byref(v)) == 0
            errs.append(v.value)
        for p in own:
            lib.eia_ar_free(ctypes.c_void_p(p))
        print(f"W={world} {'cached  ' if cached else 'uncached'} us: " + "  ".join(line) +
              f"  BAD {bad} SPIN_ERR {any(errs)}", flush=True)


if __name__ == "__main__":
    main()
