#!/bin/bash
# Decode attention, one-wave-per-item form (EIA_DECODE_WAVE): kernel tests, microbench A/B
# against the 4-wave form, and the engine-loop A/B.  First failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -x -q \
  --timeout 120 --timeout-method thread -k "decode or engine or swap" \
  > gpurun_out/wave_tests.log 2>&1 || { tail -40 gpurun_out/wave_tests.log; exit 1; }
tail -2 gpurun_out/wave_tests.log
for v in 0 1; do
  EIA_DECODE_WAVE=$v timeout -k 10 300 python scripts/bench_attn.py --batch ${BATCHES:-16 32 65 128} \
    --ctx ${CTXS:-192 1024 4096} > gpurun_out/wave_attn_$v.log 2>&1 || { tail -20 gpurun_out/wave_attn_$v.log; exit 1; }
  echo "== EIA_DECODE_WAVE=$v"; grep '"B"' gpurun_out/wave_attn_$v.log | cut -c1-110
done
VALS="0 1" bash scripts/gpu_ab.sh EIA_DECODE_WAVE "" 5
