#!/bin/bash
# Two-row-block skinny GEMM (129-256 rows): GEMM tests, 8B tables at buckets 9-16, and an engine
# decode A/B at 200 users (table before / after).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/t_gemm_rb.log 2>&1 || { tail -30 gpurun_out/t_gemm_rb.log; exit 1; }
tail -1 gpurun_out/t_gemm_rb.log
cp enterprise_inference_amd/ops/gemm_tuning.json gpurun_out/table_before_rb.json
MS="136 144 152 160 168 176 184 192 200 208 216 224 232 240 248 256"
SH=${RB_SHAPES:-qkv_8b o_8b gate_up_8b down_8b lm_head_8b}
timeout -k 10 900 python scripts/bench_gemm.py --tune --m $MS --shapes $SH \
  --out gpurun_out/gemm_tuning.json > gpurun_out/tune_rb.log 2>&1 || exit 1
timeout -k 10 900 python scripts/bench_gemm.py --tune --wgpack --m $MS --shapes $SH \
  --out gpurun_out/gemm_tuning.json > gpurun_out/tune_rb_wg.log 2>&1 || exit 1
grep -h '"bucket"' gpurun_out/tune_rb.log | cut -c1-150
R=$PWD
for t in before after; do
  tab=$R/gpurun_out/table_before_rb.json; [[ $t == after ]] && tab=$R/gpurun_out/gemm_tuning.json
  EIA_GEMM_TUNING=$tab timeout -k 10 600 python bench.py --mode engine --users ${RB_USERS:-200} \
    --steps 2 --warmup 1 > gpurun_out/rb_engine_$t.log 2>&1 || exit 1
  echo "$t $(grep '^{' gpurun_out/rb_engine_$t.log | tail -1 | cut -c1-400)"
done
