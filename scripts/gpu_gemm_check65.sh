#!/bin/bash
# Decode-GEMM tuning-table regret at the headline's M (65) and the bucket's other edge.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python scripts/bench_gemm.py --check --m 65 80 \
  --shapes qkv_8b o_8b gate_up_8b down_8b lm_head_8b 2>&1 | tee gpurun_out/gemm_check65.log
