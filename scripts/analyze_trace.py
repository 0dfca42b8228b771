#!/usr/bin/env python3
"""GPU busy/idle analysis of a rocprofv3 ``*_kernel_trace.csv``.

Reports, over the last ``--tail`` seconds of the trace (the timed bench rounds), the
kernel-busy time (union of dispatch intervals), the idle time between dispatches split
by gap size, and the kernels with the largest share.  Idle time between two kernels of a
decode step is host overhead (scheduling, metadata, sampling read-back) the GPU waits on.

Usage: analyze_trace.py <dir-or-csv> [--tail 1.5]
"""
import argparse
import collections
import csv
import glob
import os
import re
import sys


def find_csv(p: str) -> str:
    if os.path.isfile(p):
        return p
    c = glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
    if not c:
        raise SystemExit(f"no kernel_trace.csv under {p}")
    return c[0]


def short(name: str) -> str:
    if name.startswith(("Cijk_", "Custom_Cijk")):
        m = re.search(r"MT(\d+x\d+x\d+)", name)
        return f"hipBLASLt MT{m.group(1) if m else '?'}"
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)[:60]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--tail", type=float, default=1.5, help="seconds at the end of the trace")
    a = ap.parse_args()
    rows = []
    with open(find_csv(a.path)) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    t_end = max(e for _, e, _ in rows)
    t0 = t_end - int(a.tail * 1e9)
    rows = [r for r in rows if r[0] >= t0]
    busy = 0
    cur_s, cur_e = rows[0][0], rows[0][1]
    gaps = []
    for s, e, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = rows[-1][1] - rows[0][0]
    per = collections.Counter()
    cnt = collections.Counter()
    for s, e, n in rows:
        per[short(n)] += e - s
        cnt[short(n)] += 1
    print(f"window: last {a.tail:.2f}s, {len(rows)} dispatches, span {span / 1e6:.2f} ms")
    print(f"busy (union) {busy / 1e6:.2f} ms = {100 * busy / span:.1f}% ; idle {(span - busy) / 1e6:.2f} ms")
    buckets = [(0, 2e3), (2e3, 10e3), (10e3, 50e3), (50e3, 200e3), (200e3, 1e12)]
    for lo, hi in buckets:
        g = [x for x in gaps if lo <= x < hi]
        print(f"  gaps {lo / 1e3:>6.0f}-{hi / 1e3:<8.0f}us: n={len(g):6d} total {sum(g) / 1e6:8.2f} ms")
    where = collections.Counter()
    for x, y in zip(rows, rows[1:]):
        if y[0] - x[1] > 200e3:
            where[(short(x[2])[:40], short(y[2])[:40])] += 1
    if where:
        print("\nidle gaps > 200 us, by (kernel before -> kernel after):")
        for (x, y), n in where.most_common(6):
            print(f"  {n:5d}  {x} -> {y}")
    print("\n| kernel | calls | total ms | % busy | avg us |\n|---|---:|---:|---:|---:|")
    for n, t in per.most_common(25):
        print(f"| {n} | {cnt[n]} | {t / 1e6:.2f} | {100 * t / busy:.1f} | {t / cnt[n] / 1e3:.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
