#!/bin/bash
# Mixtral decode MoE: down-projection K split 2 vs 4 with the staggered K walk on (engine A/B).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for s in 2 4 2 4; do
  EIA_MOE_DOWN_SK=$s timeout -k 10 400 python bench.py --model mistralai/Mixtral-8x7B-Instruct-v0.1 --mode engine --steps 3 --warmup 1 > gpurun_out/moe_sk2_$s.log 2>&1 || exit 1
  echo "down_sk=$s $(tail -1 gpurun_out/moe_sk2_$s.log | grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' | tr '\n' ' ')"
done
