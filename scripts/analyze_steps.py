#!/usr/bin/env python3
"""Per-decode-step view of a rocprofv3 kernel trace (``*_kernel_trace.csv``).

A decode step ends at the sampler's merge kernel; the last N complete steps are averaged:
launches per step, kernel time per step, step span (first start -> last end) and the busy
fraction (kernel time / span), then the per-kernel time per step.

Usage: analyze_steps.py <kernel_trace.csv> [title] [steps] [end_kernel_substring] [last|longest]

``longest`` averages the N steps with the most kernel time instead of the last N (the prefill
steps of a burst round).
"""
import collections
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"MT(\d+x\d+x\d+)", name)
    if name.startswith(("Cijk_", "Custom_Cijk")):
        return f"hipBLASLt GEMM MT{m.group(1) if m else '?'}"
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return re.sub(r"\(.*", "", name)[:72]


def main() -> int:
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    marker = sys.argv[4] if len(sys.argv) > 4 else "sample_merge"
    pick = sys.argv[5] if len(sys.argv) > 5 else "last"
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    ends = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
    if len(ends) < 2:
        print(f"no steps found (marker {marker!r})")
        return 1
    nsteps = min(nsteps, len(ends) - 1)
    pairs = list(zip(ends[-nsteps - 1:-1], ends[-nsteps:]))
    if pick == "longest":
        def ktime(ab):
            return sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                       for r in rows[ab[0] + 1:ab[1] + 1])
        pairs = sorted(zip(ends[:-1], ends[1:]), key=ktime)[-nsteps:]
    agg = collections.defaultdict(list)
    by_grid = collections.defaultdict(list)  # (kernel, grid) -> durations: tells one GEMM shape from another
    gaps = collections.defaultdict(list)     # idle before a kernel, keyed by (previous, kernel)
    spans, busy, launches = [], [], []
    for a, b in pairs:
        ks = rows[a + 1:b + 1]
        for prev, cur in zip(ks[:-1], ks[1:]):
            g = (int(cur["Start_Timestamp"]) - int(prev["End_Timestamp"])) / 1e3
            gaps[(short(prev["Kernel_Name"])[:40], short(cur["Kernel_Name"])[:40])].append(g)
        t0 = int(ks[0]["Start_Timestamp"])
        t1 = int(ks[-1]["End_Timestamp"])
        spans.append((t1 - t0) / 1e3)
        k = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in ks) / 1e3
        busy.append(k)
        launches.append(len(ks))
        for r in ks:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            agg[short(r["Kernel_Name"])].append(d)
            grid = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
            by_grid[(short(r["Kernel_Name"])[:60], grid)].append(d)
    n = len(pairs)
    span, kern = sum(spans) / n, sum(busy) / n
    print(f"### {title}\n")
    print(f"{'Last' if pick != 'longest' else 'Longest'} {n} steps: {sum(launches) / n:.0f} launches/step, kernel time "
          f"{kern / 1e3:.3f} ms/step, span {span / 1e3:.3f} ms/step, busy {100 * kern / span:.1f} %\n")
    print("| kernel | launches/step | µs/step | % of kernel time | avg µs |")
    print("|---|---:|---:|---:|---:|")
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        per = sum(v) / n
        print(f"| {name} | {len(v) / n:.1f} | {per:.1f} | {100 * per / kern:.1f} | {sum(v) / len(v):.2f} |")
    print("\nBy kernel and grid (threads x, y, z): one row per GEMM shape / launch form:\n")
    print("| kernel | grid | launches/step | avg us | us/step |")
    print("|---|---|---:|---:|---:|")
    for (name, grid), v in sorted(by_grid.items(), key=lambda kv: -sum(kv[1]))[:24]:
        print(f"| {name} | {grid} | {len(v) / n:.1f} | {sum(v) / len(v):.2f} | {sum(v) / n:.1f} |")
    # one step's copies and their neighbours, relative times (us)
    a, b = pairs[len(pairs) // 2]
    seq = rows[a - 2:b + 3]
    base = int(seq[0]["Start_Timestamp"])
    print("\nA middle step around the staging copies (us from the first row):\n")
    print("| # | kernel | start | end | gap before |")
    print("|---:|---|---:|---:|---:|")
    prev_end = None
    for i, r in enumerate(seq):
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        nm = short(r["Kernel_Name"])
        near = any("copyBuffer" in short(x["Kernel_Name"]) for x in seq[max(0, i - 2):i + 3])
        if near or i < 3 or i > len(seq) - 4:
            gap = "" if prev_end is None else f"{(st - prev_end) / 1e3:.2f}"
            print(f"| {i} | {nm[:48]} | {(st - base) / 1e3:.2f} | {(en - base) / 1e3:.2f} | {gap} |")
        prev_end = en
    print("\nIdle between consecutive kernels (by pair; us per step = count x mean gap):\n")
    print("| previous -> next | per step | mean gap us | us/step |")
    print("|---|---:|---:|---:|")
    for (pa, pb), v in sorted(gaps.items(), key=lambda kv: -sum(kv[1]))[:14]:
        print(f"| {pa} -> {pb} | {len(v) / n:.1f} | {sum(v) / len(v):.2f} | {sum(v) / n:.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
