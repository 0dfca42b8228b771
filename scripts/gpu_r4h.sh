#!/bin/bash
# Stream-K merge in one round trip + wide add+norm without fences: numerics, attention
# microbench (short and long context, more partition counts), engine A/B per feature.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py::test_splitk_add_rmsnorm tests/test_kernels_gpu.py -k "decode_sk or splitk_add" \
  > gpurun_out/pytest_r4h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r4h.log; [[ $rc != 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_attn.py --batch 16 64 65 --ctx 192 --fused-sk 4 --p-only 1 --flush-mb 512 > gpurun_out/attn_sk2.log 2>&1
rc=$?; cut -c1-330 gpurun_out/attn_sk2.log | grep '"B"'; [[ $rc != 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_attn.py --batch 35 --ctx 2048 4096 --p-only 1 2 3 4 6 8 16 --flush-mb 512 > gpurun_out/attn_long2.log 2>&1
rc=$?; cut -c1-500 gpurun_out/attn_long2.log | grep '"B"'; [[ $rc != 0 ]] && exit $rc
for v in "0 0" "0 1" "1 0"; do
  set -- $v
  EIA_DECODE_SK=$1 EIA_ADDNORM_WIDE=$2 timeout -k 10 400 python bench.py --mode engine --steps 3 --warmup 1 > gpurun_out/eng_$1$2.log 2>&1 || exit 1
  echo "SK=$1 WIDE=$2 $(tail -1 gpurun_out/eng_$1$2.log | grep -o '"tpot_p50_ms": [0-9.]*')"
done
EIA_FA_IL=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k prefill > gpurun_out/pytest_fa3.log 2>&1
rc=$?; echo "FA_IL=3 tests: $(tail -1 gpurun_out/pytest_fa3.log)"; [[ $rc != 0 ]] && exit $rc
for il in 0 1 2 3; do
  EIA_FA_IL=$il timeout -k 10 200 python scripts/bench_prefill_attn.py --shapes 1x8192 4x2048 65x128 --qt 32 > gpurun_out/fa_il$il.log 2>&1 || exit 1
  echo "FA_IL=$il"; grep -o '"shape": "[0-9x]*".*"tflops": [0-9.]*' gpurun_out/fa_il$il.log | sed 's/"causal.*"us"/ us/'
done
PMC_TAG=_r4 bash scripts/gpu_pmc_prefill.sh > gpurun_out/pmc_prefill_r4.log 2>&1
rc=$?; tail -6 gpurun_out/pmc_prefill_r4.log; exit $rc
