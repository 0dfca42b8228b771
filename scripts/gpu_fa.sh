#!/bin/bash
# prefill attention: GPU kernel tests (-k prefill) then the FA microbench (causal + non-causal)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out; export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "prefill" > gpurun_out/fa_tests.log 2>&1 || { tail -30 gpurun_out/fa_tests.log; exit 1; }
tail -1 gpurun_out/fa_tests.log
timeout -k 10 300 python scripts/bench_prefill_attn.py --shapes ${FA_SHAPES:-1x8192 4x2048 16x512} \
  > gpurun_out/fa_bench.log 2>&1 || { tail -20 gpurun_out/fa_bench.log; exit 1; }
timeout -k 10 120 python scripts/bench_prefill_attn.py --shapes 1x8192 --noncausal \
  >> gpurun_out/fa_bench.log 2>&1 || { tail -20 gpurun_out/fa_bench.log; exit 1; }
cat gpurun_out/fa_bench.log
