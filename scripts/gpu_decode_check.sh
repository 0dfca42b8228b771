#!/bin/bash
# Decode-attention change check: GPU kernel/e2e tests selected by -k, then the per-step rocprofv3
# decode profile of the engine loop for each EIA_DECODE_WAVE value.  First failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${KEXPR:-decode or rope or attention or engine or e2e or swap or canary}" \
  > gpurun_out/dc_tests.log 2>&1 || { tail -40 gpurun_out/dc_tests.log; exit 1; }
tail -2 gpurun_out/dc_tests.log
VALS="${WAVES:-0 1}" bash scripts/gpu_prof_ab.sh EIA_DECODE_WAVE
