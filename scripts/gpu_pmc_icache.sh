#!/bin/bash
# Instruction-cache counters for the decode attention microbench (fused RoPE form, B 65,
# ctx 192, P 1, cold Infinity Cache): is the short-lived straight-line kernel fetch-bound?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=$R/gpurun_out/pmc_icache
mkdir -p "$OUT"
cd /tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
grep -o "SQC_[A-Z_]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_]*\|SQ_WAIT_[A-Z_]*" "$OUT/avail.txt" | sort -u | tr '\n' ' ' > "$OUT/names.txt"
cat "$OUT/names.txt"; echo
C=${COUNTERS:-SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU}
timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $C -d "$OUT/p1" -o run --output-format csv -- \
  python3 "$R/scripts/bench_attn.py" --batch 65 --ctx 192 --p-only 1 --fused-sk 4 --flush-mb 512 \
  > "$OUT/log1.txt" 2>&1 || { tail -5 "$OUT/log1.txt"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
f = glob.glob(f"{out}/p1/**/*counter_collection.csv", recursive=True)
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f[0])):
    k = r["Kernel_Name"][:70]
    if "paged_decode" not in k:
        continue
    agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
