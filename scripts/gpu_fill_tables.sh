#!/bin/bash
# Fill decode-table buckets a shape was never tuned at (scripts/bench_gemm.py --tune, plain then
# workgroup-packed).  usage: M="88 96 ..." bash scripts/gpu_fill_tables.sh SHAPE...
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-fill}
timeout -k 10 900 python scripts/bench_gemm.py --tune --m $M --shapes "$@" \
  --out gpurun_out/gemm_tuning.json > gpurun_out/tune_$TAG.log 2>&1 || exit 1
timeout -k 10 900 python scripts/bench_gemm.py --tune --wgpack --m $M --shapes "$@" \
  --out gpurun_out/gemm_tuning.json > gpurun_out/tune_${TAG}_wg.log 2>&1 || exit 1
grep -h '"bucket"' gpurun_out/tune_$TAG.log gpurun_out/tune_${TAG}_wg.log | cut -c1-160
