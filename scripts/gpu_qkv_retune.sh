#!/bin/bash
# Re-tune the QKV decode tables now that split-K past the attention's LDS staging is timed with
# its reduce launch (scripts/bench_gemm.py "defer"), then trace the TP8-rank decode step.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
S=${QKV_SHAPES:-qkv_70b_tp8 qkv_8b}
cp enterprise_inference_amd/ops/gemm_tuning.json gpurun_out/table_before_qkv.json
timeout -k 10 600 python scripts/bench_gemm.py --tune --m 33 40 48 65 72 80 --shapes $S \
  --out gpurun_out/gemm_tuning.json > gpurun_out/tune_qkv.log 2>&1 || exit 1
timeout -k 10 600 python scripts/bench_gemm.py --tune --wgpack --m 33 40 48 65 72 80 --shapes $S \
  --out gpurun_out/gemm_tuning.json > gpurun_out/tune_qkv_wg.log 2>&1 || exit 1
grep -h '"bucket"' gpurun_out/tune_qkv.log gpurun_out/tune_qkv_wg.log
