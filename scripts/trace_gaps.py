#!/usr/bin/env python3
"""GPU idle gaps in a rocprofv3 kernel trace window (where a step's wall time is not kernels).

  python scripts/trace_gaps.py run_kernel_trace.csv --after-gap-ms 20 --window-ms 120

Finds the last idle gap of at least --after-gap-ms (the host-side pause before a traced round,
e.g. scripts/burst_timeline.py's synchronize between its warm and traced rounds), then lists
from the first kernel after it, over --window-ms: kernel time, busy share, the idle gaps of at
least --min-gap-us with the kernels on either side, and kernel time by name.
"""
from __future__ import annotations

import argparse
import collections
import csv


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--after-gap-ms", type=float, default=20.0)
    ap.add_argument("--window-ms", type=float, default=120.0)
    ap.add_argument("--min-gap-us", type=float, default=50.0)
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    start_i = 0
    end_so_far = rows[0][1]
    for i in range(1, len(rows)):
        if rows[i][0] - end_so_far >= a.after_gap_ms * 1e6:
            start_i = i
        end_so_far = max(end_so_far, rows[i][1])
    t0 = rows[start_i][0]
    win = [r for r in rows[start_i:] if r[0] - t0 <= a.window_ms * 1e6]
    busy = 0
    cur_end = t0
    gaps = []
    by_name = collections.defaultdict(lambda: [0, 0.0])
    prev_name = None
    for s, e, n in win:
        if s > cur_end:
            g = s - cur_end
            if g >= a.min_gap_us * 1e3:
                gaps.append(((cur_end - t0) / 1e6, g / 1e3, prev_name, n))
            busy += e - s
        else:
            busy += max(0, e - cur_end)
        cur_end = max(cur_end, e)
        prev_name = n
        by_name[n[:90]][0] += 1
        by_name[n[:90]][1] += (e - s) / 1e3
    span = (cur_end - t0) / 1e6
    print(f"window: {len(win)} kernels, span {span:.2f} ms, busy {busy / 1e6:.2f} ms "
          f"({100 * busy / max(1, cur_end - t0):.1f} %)")
    print(f"\nidle gaps >= {a.min_gap_us} us: {len(gaps)}, total {sum(g[1] for g in gaps) / 1e3:.2f} ms")
    for at, g, p, n in gaps[:60]:
        print(f"  at {at:8.3f} ms  gap {g:8.1f} us  after {str(p)[:60]}  before {n[:60]}")
    print("\nkernel time by name:")
    for n, (c, us) in sorted(by_name.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"  {us / 1e3:8.3f} ms  {c:5d}x  {n}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
