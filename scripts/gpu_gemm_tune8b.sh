#!/bin/bash
# Llama-3.1-8B decode GEMMs: re-tune every 16-row bucket on three rows each (bucket edges + middle)
# and measure the table's regret at rows between the tuned ones, before and after.
#   bash scripts/gpu_gemm_tune8b.sh before|tune|after
set -eo pipefail
mkdir -p gpurun_out
S="qkv_8b o_8b gate_up_8b down_8b lm_head_8b"
CHK="12 28 44 60 76 92 108 124"
case "$1" in
  before) timeout -k 10 900 python scripts/bench_gemm.py --check --m $CHK --shapes $S 2>&1 \
            | tee gpurun_out/gemm8b_check_before.log ;;
  tune)   timeout -k 10 1000 python scripts/bench_gemm.py --tune --shapes $S \
            --m 1 8 16 17 24 32 33 40 48 49 56 64 65 72 80 81 88 96 97 104 112 113 120 128 \
            --out gpurun_out/tune8b.json 2>&1 | tee gpurun_out/tune8b.log ;;
  after)  timeout -k 10 900 python scripts/bench_gemm.py --check --m $CHK --shapes $S 2>&1 \
            | tee gpurun_out/gemm8b_check_after.log ;;
esac
