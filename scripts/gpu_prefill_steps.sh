#!/bin/bash
# Engine-loop kernel trace of the headline model: the longest (prefill) steps and the decode steps.
#   MODEL=... TAG=... bash scripts/gpu_prefill_steps.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
MODEL=${MODEL:-meta-llama/Llama-3.1-8B-Instruct}
TAG=${TAG:-8b}
OUT=$R/gpurun_out/prof_pf_$TAG
mkdir -p "$OUT"
( cd /tmp && timeout -k 10 ${LIMIT:-600} rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv \
    -- python3 "$R/bench.py" --mode engine --model "$MODEL" --steps 2 --warmup 1 ) \
    > "gpurun_out/prof_pf_$TAG.log" 2>&1 || { tail -20 "gpurun_out/prof_pf_$TAG.log"; exit 1; }
CSV=$(find "$OUT" -name '*kernel_trace.csv' | head -1)
python3 scripts/analyze_steps.py "$CSV" "$MODEL prefill" 3 sample_merge longest > "gpurun_out/prefill_steps_$TAG.md" 2>&1 || true
python3 - "$CSV" > "gpurun_out/prefill_gemm_names_$TAG.txt" <<'PY' || true
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
c = collections.defaultdict(list)
for r in rows:
    n = r["Kernel_Name"]
    if n.startswith(("Cijk_", "Custom_Cijk")) or "act_and_mul" in n or "prefill" in n:
        g = "x".join(r.get(k, "?") for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"))
        c[(n[:120], g)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (n, g), v in sorted(c.items(), key=lambda kv: -sum(kv[1]))[:30]:
    print(len(v), "avg_us %.1f" % (sum(v) / len(v)), "grid", g, n)
PY
rm -f "$CSV"
head -30 "gpurun_out/prefill_steps_$TAG.md"
