#!/bin/bash
# Prefill flash attention (raw exp2, branch-free mask, tree reductions, static priority) and the
# full-chip split-K add+RMSNorm: numerics, then the prefill microbench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py::test_splitk_add_rmsnorm tests/test_kernels_gpu.py -k "prefill or splitk_add" \
  > gpurun_out/pytest_r4e.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_r4e.log; [[ $rc != 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_prefill_attn.py --shapes 1x8192 4x2048 16x512 65x128 > gpurun_out/prefill_r4e.log 2>&1
rc=$?; cut -c1-300 gpurun_out/prefill_r4e.log; exit $rc
