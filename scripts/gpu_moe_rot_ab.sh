#!/bin/bash
# Mixtral decode MoE: staggered K walk in the grouped expert GEMMs (EIA_MOE_ROT) -- numerics,
# microbench and engine A/B on one box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
EIA_MOE_ROT=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_moe_gpu.py > gpurun_out/pytest_moe_rot.log 2>&1
rc=$?; tail -1 gpurun_out/pytest_moe_rot.log; [[ $rc != 0 ]] && exit $rc
for r in 0 3 0 3 1 5; do
  EIA_MOE_ROT=$r timeout -k 10 200 python scripts/bench_moe.py --tokens 65 --iters 20 > gpurun_out/moe_rot_mb$r.log 2>&1 || exit 1
  echo "rot=$r $(grep '^{' gpurun_out/moe_rot_mb$r.log | tail -1 | cut -c1-260)"
done
for r in 0 3 0 3; do
  EIA_MOE_ROT=$r timeout -k 10 400 python bench.py --model mistralai/Mixtral-8x7B-Instruct-v0.1 --mode engine --steps 3 --warmup 1 > gpurun_out/moe_rot$r.log 2>&1 || exit 1
  echo "engine rot=$r $(tail -1 gpurun_out/moe_rot$r.log | grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' | tr '\n' ' ')"
done
