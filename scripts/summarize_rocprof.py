#!/usr/bin/env python3
"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a markdown table.

Usage: summarize_rocprof.py <kernel_stats.csv> [title] [top_n]
Kernel names are shortened (hipBLASLt Tensile names -> their macro-tile).
"""
import csv
import re
import sys


def short(name: str) -> str:
    m = re.search(r"MT(\d+x\d+x\d+)", name)
    if name.startswith(("Cijk_", "Custom_Cijk")):
        return f"hipBLASLt GEMM MT{m.group(1) if m else '?'}"
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    return name[:70]


def main() -> int:
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"### {title}\n")
    print(f"Total GPU kernel time: {tot / 1e6:.1f} ms over {sum(int(r['Calls']) for r in rows)} launches\n")
    print("| kernel | calls | total ms | % | avg µs |")
    print("|---|---:|---:|---:|---:|")
    for r in rows[:top]:
        print(f"| {short(r['Name'])} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
              f"{float(r['Percentage']):.2f} | {float(r['AverageNs']) / 1e3:.1f} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
