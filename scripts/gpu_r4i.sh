#!/bin/bash
# Wide add+RMSNorm with batched last-arriver loads: numerics + engine A/B; prefill FA tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gemm_gpu.py::test_splitk_add_rmsnorm tests/test_kernels_gpu.py -k "prefill or splitk_add" \
  > gpurun_out/pytest_r4i.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r4i.log; [[ $rc != 0 ]] && exit $rc
for v in 0 1 0 1; do
  EIA_ADDNORM_WIDE=$v timeout -k 10 400 python bench.py --mode engine --steps 3 --warmup 1 > gpurun_out/eng_w$v.log 2>&1 || exit 1
  echo "WIDE=$v $(tail -1 gpurun_out/eng_w$v.log | grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' | tr '\n' ' ')"
done
timeout -k 10 200 python scripts/bench_prefill_attn.py --shapes 1x8192 4x2048 16x512 65x128 --qt 32 > gpurun_out/fa_r4i.log 2>&1
rc=$?; grep -o '"shape": "[0-9x]*".*"tflops": [0-9.]*' gpurun_out/fa_r4i.log | sed 's/"causal.*"us"/ us/'; exit $rc
