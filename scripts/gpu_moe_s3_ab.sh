#!/bin/bash
# Mixtral decode MoE: 3-stage weight pipeline in the grouped expert GEMMs (EIA_MOE_UP_CFG=7,
# EIA_MOE_DOWN_CFG=6) vs the 2-stage defaults (3 / 2) -- microbench and engine A/B on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run_mb() {  # tag up down
  EIA_MOE_UP_CFG=$2 EIA_MOE_DOWN_CFG=$3 timeout -k 10 200 python scripts/bench_moe.py --tokens 65 33 --iters 20 > gpurun_out/moe_s3_$1.log 2>&1 || return 1
  echo "$1 up=$2 down=$3"; grep '^{' gpurun_out/moe_s3_$1.log | cut -c1-200
}
run_mb a 3 2 && run_mb b 7 6 && run_mb c 3 6 && run_mb d 7 2 && run_mb e 3 2 && run_mb f 7 6 || exit 1
for v in "3 2" "7 6" "3 2" "7 6"; do
  set -- $v
  EIA_MOE_UP_CFG=$1 EIA_MOE_DOWN_CFG=$2 timeout -k 10 400 python bench.py --model mistralai/Mixtral-8x7B-Instruct-v0.1 --mode engine --steps 3 --warmup 1 > gpurun_out/moe_s3_eng.log 2>&1 || exit 1
  echo "engine up=$1 down=$2 $(tail -1 gpurun_out/moe_s3_eng.log | grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' | tr '\n' ' ')"
done
