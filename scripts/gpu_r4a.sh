#!/bin/bash
# Round-4 first GPU session: the GPU test suite on the cleaned tree, then the endpoint HIP-API
# trace of the decode loop (which host call sits in the step-boundary idle).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; [[ $rc != 0 ]] && exit $rc
MODE=endpoint NGAPS=8 LOOKBACK_MS=5 bash scripts/gpu_api_trace.sh
rc=$?; tail -3 gpurun_out/api.log; head -60 gpurun_out/api_gaps.txt; exit $rc
