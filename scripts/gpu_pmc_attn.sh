#!/bin/bash
# PMC counters for the decode attention microbench (kernel-trace + counters only), B 32 / 65
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=$R/gpurun_out/pmc_attn
mkdir -p "$OUT"
cd /tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA FETCH_SIZE \
  -d "$OUT/p1" -o run --output-format csv -- python3 "$R/scripts/bench_attn.py" --batch 32 65 --ctx 192 \
  > "$OUT/log1.txt" 2>&1 || { tail -5 "$OUT/log1.txt"; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_INSTS_SALU SQ_WAIT_INST_LDS TA_BUSY_avr GRBM_GUI_ACTIVE \
  -d "$OUT/p2" -o run --output-format csv -- python3 "$R/scripts/bench_attn.py" --batch 32 65 --ctx 192 \
  > "$OUT/log2.txt" 2>&1 || { tail -5 "$OUT/log2.txt"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for p in ("p1", "p2"):
    f = glob.glob(f"{out}/{p}/**/*counter_collection.csv", recursive=True)
    if not f:
        print("no counters", p); continue
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    grid = {}
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"][:60]
        if "paged_decode" not in k:
            continue
        key = (k, r.get("Grid_Size", ""))
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for key, d in agg.items():
        print(p, key, {c: round(sum(v) / len(v)) for c, v in d.items()})
PY
