#!/bin/bash
# Mixtral decode MoE: down projection split over K (EIA_MOE_DOWN_SK) -- numerics, engine A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py > gpurun_out/pytest_moe.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_moe.log; [[ $rc != 0 ]] && exit $rc
for s in 1 2 4 1 2 4; do
  EIA_MOE_DOWN_SK=$s timeout -k 10 400 python bench.py --model mistralai/Mixtral-8x7B-Instruct-v0.1 --mode engine --steps 3 --warmup 1 > gpurun_out/moe_sk$s.log 2>&1 || exit 1
  echo "down_sk=$s $(tail -1 gpurun_out/moe_sk$s.log | grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' | tr '\n' ' ')"
done
