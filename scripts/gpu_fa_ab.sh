#!/bin/bash
# Prefill flash attention A/B on one box: env flag $AB_FLAG 0 / 1, alternating, two pairs
# (AB_FLAG default EIA_FA_ASM_ADD); kernel tests first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
F=${AB_FLAG:-EIA_FA_ASM_ADD}
for v in 0 1; do
  env $F=$v timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "prefill" > gpurun_out/fa_tests_$v.log 2>&1 || { tail -30 gpurun_out/fa_tests_$v.log; exit 1; }
  tail -1 gpurun_out/fa_tests_$v.log
done
: > gpurun_out/fa_ab.log
for pass in 1 2; do
  for v in 0 1; do
    echo "== $F=$v pass $pass" >> gpurun_out/fa_ab.log
    env $F=$v timeout -k 10 300 python scripts/bench_prefill_attn.py --shapes ${FA_SHAPES:-1x8192 4x2048 16x512} \
      >> gpurun_out/fa_ab.log 2>&1 || { tail -20 gpurun_out/fa_ab.log; exit 1; }
    env $F=$v timeout -k 10 120 python scripts/bench_prefill_attn.py --shapes 1x8192 --noncausal \
      >> gpurun_out/fa_ab.log 2>&1 || { tail -20 gpurun_out/fa_ab.log; exit 1; }
  done
done
cat gpurun_out/fa_ab.log
