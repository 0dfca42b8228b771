#!/bin/bash
# Llama-3.3-70B one-GPU decode GEMMs: re-tune buckets 1-5 on three rows each, one step per shape
# (each step reads the table the previous one wrote).  Writes gpurun_out/tune70x3_<shape>.{log,json}.
#   bash scripts/gpu_gemm_tune70x3.sh qkv_70b o_70b ...
set -eo pipefail
mkdir -p gpurun_out
for s in "$@"; do
  timeout -k 10 1000 python scripts/bench_gemm.py --tune --shapes "$s" \
    --m 1 8 16 17 24 32 33 40 48 49 56 64 65 72 80 \
    --out "gpurun_out/tune70x3_$s.json" 2>&1 | tee "gpurun_out/tune70x3_$s.log"
done
