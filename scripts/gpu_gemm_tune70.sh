#!/bin/bash
# Fill the 70B tuning-table buckets that were never timed (one-GPU gate_up / lm_head at 17-32 and
# 49-64 rows; the TP4 shard shapes at 1-16, 17-32 and 49-64 rows).  Writes gpurun_out/tune70*.json;
# merge the new keys into enterprise_inference_amd/ops/gemm_tuning.json by hand.
set -eo pipefail
mkdir -p gpurun_out
timeout -k 10 600 python scripts/bench_gemm.py --tune --m 24 56 --shapes gate_up_70b lm_head_70b \
  --out gpurun_out/tune70_tp1.json 2>&1 | tee gpurun_out/tune70_tp1.log
timeout -k 10 600 python scripts/bench_gemm.py --tune --m 8 24 56 \
  --shapes qkv_70b_tp4 o_70b_tp4 gate_up_70b_tp4 down_70b_tp4 lm_head_70b_tp4 \
  --out gpurun_out/tune70_tp4.json 2>&1 | tee gpurun_out/tune70_tp4.log
