#!/bin/bash
# Sizing-guide rows through the endpoint on one GPU (reference third_party/IBM/docs/
# sizing-guide.md:56-63 for 8b, :69-76 for 70b), a few cases per box call:
#   bash scripts/gpu_sizing.sh MODEL TAG [case ...]      (MODEL: 8b | 70b)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MODEL=$1; TAG=$2; shift 2
PER=$([[ "$MODEL" == 70b ]] && echo 540 || echo 400)
timeout -k 10 1150 python scripts/sizing_sweep.py --model "$MODEL" ${*:+--cases "$@"} \
  --timeout "$PER" --out "gpurun_out/sizing_${MODEL}_$TAG.md" 2>&1 \
  | tee "gpurun_out/sizing_${MODEL}_$TAG.log"
rc=$?; cat "gpurun_out/sizing_${MODEL}_$TAG.md"; exit $rc
