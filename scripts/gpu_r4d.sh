#!/bin/bash
# Stream-K decode attention: kernel tests, microbench vs the fused per-item kernel, engine A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "decode_sk or decode_rope_fused" --timeout 120 --timeout-method thread > gpurun_out/pytest_sk.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_sk.log; [[ $rc != 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_attn.py --batch 16 32 64 65 96 --ctx 192 256 1024 --fused-sk 4 --p-only 1 2 --flush-mb 512 > gpurun_out/attn_sk.log 2>&1
rc=$?; cut -c1-250 gpurun_out/attn_sk.log | grep '"B"'; [[ $rc != 0 ]] && exit $rc
timeout -k 10 300 python scripts/bench_attn.py --batch 35 --ctx 2048 4096 --fused-sk 4 --p-only 1 2 --flush-mb 512 > gpurun_out/attn_long.log 2>&1
rc=$?; cut -c1-250 gpurun_out/attn_long.log | grep '"B"'; [[ $rc != 0 ]] && exit $rc
for v in 0 1; do
  EIA_ADDNORM_WIDE=$v EIA_DECODE_SK=$v timeout -k 10 400 python bench.py --mode engine --steps 3 --warmup 1 > gpurun_out/eng_sk$v.log 2>&1 || exit 1
  echo "EIA_DECODE_SK=EIA_ADDNORM_WIDE=$v"; tail -1 gpurun_out/eng_sk$v.log | cut -c1-400
done
