#!/bin/bash
# Stream-K decode failure census (every case, no -x) + prefill FA (two-tile-ahead K/V fetch).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "prefill" -x > gpurun_out/pytest_fa.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_fa.log; [[ $rc != 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_prefill_attn.py --shapes 1x8192 4x2048 16x512 65x128 --qt 32 \
  > gpurun_out/prefill_r4g.log 2>&1
rc=$?; cut -c1-200 gpurun_out/prefill_r4g.log; [[ $rc != 0 ]] && exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "decode_sk" -rf > gpurun_out/pytest_sk.log 2>&1
rc=$?; grep -E "^FAILED|^E  .*(differ|mismatch|max|Assertion)|passed|failed" gpurun_out/pytest_sk.log | cut -c1-400 | head -40
exit $rc
