#!/usr/bin/env python3
"""Correlate GPU idle gaps (kernel trace) with host HIP API calls (hip trace) on the same
clock: for the largest gaps, print the API calls issued from 1.5 ms before the gap until its
end, so a late launch can be attributed to the host call that was blocking.

Usage: analyze_api_gaps.py <rocprofv3 output dir> [--n 3]
"""
import argparse
import csv
import glob
import os
import re


def load(d, pat):
    f = glob.glob(os.path.join(d, "**", pat), recursive=True)
    if not f:
        raise SystemExit(f"no {pat} under {d}")
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def short(n):
    n = n.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", n)[:50]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--n", type=int, default=3)
    ap.add_argument("--min-gap-us", type=float, default=200)
    ap.add_argument("--lookback-ms", type=float, default=1.5)
    a = ap.parse_args()
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
                for r in load(a.path, "*kernel_trace.csv"))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                  r["Function"] + " [tid %s]" % r.get("Thread_Id", "?"))
                 for r in load(a.path, "*hip_api_trace.csv"))
    try:
        for r in load(a.path, "*memory_copy_trace.csv"):
            ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                       "memcpy " + r.get("Direction", "?")))
        ks.sort()
    except SystemExit:
        pass
    gaps = [(ks[i][0] - ks[i - 1][1], ks[i - 1][1], ks[i][0], ks[i - 1][2], ks[i][2])
            for i in range(1, len(ks)) if ks[i][0] - ks[i - 1][1] > a.min_gap_us * 1e3]
    print(f"{len(gaps)} gaps > {a.min_gap_us} us; showing the last {a.n}")
    # how long the host spends inside each graph launch (a launch that blocks until the GPU
    # has nearly drained serialises the host behind every step)
    gl = sorted((t1 - t0) / 1e3 for t0, t1, f in api if f.startswith("hipGraphLaunch"))
    if gl:
        print(f"hipGraphLaunch: {len(gl)} calls, host us min {gl[0]:.1f} p50 {gl[len(gl) // 2]:.1f} "
              f"p90 {gl[int(0.9 * (len(gl) - 1))]:.1f} max {gl[-1]:.1f}")
    for g, s, e, kb, ka in gaps[-a.n:]:
        print(f"\n=== gap {g / 1e3:.1f} us: {short(kb)} -> {short(ka)}")
        for t0, t1, f in api:
            if s - a.lookback_ms * 1e6 <= t0 <= e:
                print(f"  {(t0 - s) / 1e3:9.1f} .. {(t1 - s) / 1e3:9.1f} us  {f}")


if __name__ == "__main__":
    main()
