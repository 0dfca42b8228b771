#!/bin/bash
# 7-wave SwiGLU (cfg 273): GEMM GPU tests, then 70B gate_up microbench (tuned cfg vs 273)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/g7_tests.log 2>&1 || { tail -30 gpurun_out/g7_tests.log; exit 1; }
tail -1 gpurun_out/g7_tests.log
timeout -k 10 400 python scripts/bench_gemm.py --sweep --m 17 35 48 64 --shapes gate_up_70b gate_up_8b \
  > gpurun_out/g7_gemm.log 2>&1 || { tail -20 gpurun_out/g7_gemm.log; exit 1; }
grep '"shape"' gpurun_out/g7_gemm.log | cut -c1-260
