#!/bin/bash
# Endpoint HIP-API trace of the decode loop (which host call sits in the step-boundary idle),
# then the rest of the GPU tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
MODE=endpoint NGAPS=8 LOOKBACK_MS=5 bash scripts/gpu_api_trace.sh
rc=$?; tail -3 gpurun_out/api.log; head -40 gpurun_out/api_gaps.txt; [[ $rc != 0 ]] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; exit $rc
