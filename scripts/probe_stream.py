#!/usr/bin/env python3
"""HBM read-stream probe: chip TB/s of one read pass over `--mb` megabytes (cold: a 1 GB
buffer rotated so the Infinity Cache never holds the bytes) by access shape and loads in
flight per wave (scripts/probe_stream.hip; build it first with --build on the build host).

  wg-contig   one sequential stream per workgroup (waves interleaved at 1 KiB)
  wave-contig four streams per workgroup
  rows-N      the decode GEMM's shape: each wave owns 16*N rows of 8 KiB, reads 16 rows x 64 B
              per instruction (N = 2: one SwiGLU pair / two 16-row tiles per wave)
  packed-N    the same bytes tile-packed (each 16-row tile contiguous, 1 KiB per instruction)
  *-rot       the K walk of workgroup b starts at step 3b (gemm_skinny's staggered walk)
"""
import argparse
import ctypes
import os
import statistics
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "libeia_probe_stream.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--mb", type=int, default=224)
    ap.add_argument("--wgs", type=int, nargs="*", default=[224, 256, 512])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--modes", nargs="*", default=["wg-contig", "rows-2", "rows-2-rot",
                                                   "packed-2", "packed-2-rot"])
    ap.add_argument("--u", type=int, nargs="*", default=[4, 8, 16, 32])
    a = ap.parse_args()
    table = {"wg-contig": (0, 0, 0), "wave-contig": (1, 0, 0), "rows-1": (2, 1, 0),
             "rows-2": (2, 2, 0), "rows-2-rot": (2, 2, 3), "packed-1": (3, 1, 0),
             "packed-2": (3, 2, 0), "packed-2-rot": (3, 2, 3)}
    a.modes_list = [(table[m][0], m, table[m][1], table[m][2]) for m in a.modes]
    if a.build:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC",
                        os.path.join(HERE, "probe_stream.hip"), "-o", SO], check=True)
        print("built", SO)
        return
    import torch
    lib = ctypes.CDLL(SO)
    lib.probe_stream.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_long, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
    total = 1 << 30
    buf = torch.randint(0, 255, (total,), dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4096 * 256, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    nbytes = a.mb << 20
    for wgs in a.wgs:
        for mode, name, ntile, rot in a.modes_list:
            row_bytes = 8192
            if mode >= 2:
                rows = 4 * 16 * ntile
                per_wg = rows * row_bytes
            else:
                per_wg = (nbytes // wgs) // 16384 * 16384
            used = per_wg * wgs
            if used > total // 4:
                continue
            for U in a.u:
                if mode >= 2 and U % ntile:
                    continue
                ts = []
                for it in range(a.iters):
                    off = (it % 4) * (total // 4)
                    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
                    e0.record()
                    rc = lib.probe_stream(buf.data_ptr() + off, per_wg, wgs, mode, row_bytes,
                                          ntile, U, rot, sink.data_ptr(), st)
                    e1.record()
                    e1.synchronize()
                    assert rc == 0
                    if it >= 2:
                        ts.append(e0.elapsed_time(e1) * 1e3)
                t = statistics.median(ts)
                print(f"wgs {wgs:4d} {name:12s} U {U:2d}  {used / 1e6:7.1f} MB  {t:7.2f} us  "
                      f"{used / t / 1e6:5.2f} TB/s  ({used / wgs / t / 1e3:5.1f} GB/s per WG)",
                      flush=True)


if __name__ == "__main__":
    sys.exit(main())
