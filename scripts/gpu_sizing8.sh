#!/bin/bash
# 8B single-GPU sizing rows (sizing-guide.md:56-63): bash scripts/gpu_sizing8.sh TAG [case ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=$1; shift
timeout -k 10 1150 python scripts/sizing_sweep.py --model 8b ${*:+--cases "$@"} --timeout 400 \
  --out gpurun_out/sizing_8b_$TAG.md 2>&1 | tee gpurun_out/sizing_8b_$TAG.log
rc=$?; cat gpurun_out/sizing_8b_$TAG.md; exit $rc
