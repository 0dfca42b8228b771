#!/bin/bash
# 70B single-GPU sizing rows (sizing-guide.md:69-76), a few cases per box call:
#   bash scripts/gpu_sizing70.sh TAG case [case ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=$1; shift
timeout -k 10 1150 python scripts/sizing_sweep.py --model 70b --cases "$@" --timeout 540 \
  --out gpurun_out/sizing_70b_$TAG.md 2>&1 | tee gpurun_out/sizing_70b_$TAG.log
rc=$?; cat gpurun_out/sizing_70b_$TAG.md; exit $rc
