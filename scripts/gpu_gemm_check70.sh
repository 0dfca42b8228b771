#!/bin/bash
# Decode-GEMM tuning-table regret for Llama-3.3-70B on one GPU at the sizing guide's user counts.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python scripts/bench_gemm.py --check --m ${GEMM_M:-35 60} \
  --shapes ${GEMM_SHAPES:-qkv_70b o_70b gate_up_70b down_70b lm_head_70b} 2>&1 | tee gpurun_out/gemm_check70.log
