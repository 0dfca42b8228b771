#!/bin/bash
# Engine-loop A/B of two decode GEMM tables (EIA_GEMM_TUNING): OLD=path NEW=path, then the
# per-step profile with NEW.  First failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for t in $OLD $NEW $OLD $NEW; do
  EIA_GEMM_TUNING=$t timeout -k 10 600 python bench.py --mode engine --steps 3 --warmup 1 \
    > gpurun_out/tab_ab.log 2>&1 || { tail -20 gpurun_out/tab_ab.log; exit 1; }
  echo "$t $(grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' gpurun_out/tab_ab.log | tr '\n' ' ')"
done
EIA_GEMM_TUNING=$NEW VALS="1" bash scripts/gpu_prof_ab.sh EIA_TABLE_NEW
