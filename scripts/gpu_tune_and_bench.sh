#!/bin/bash
# Tune the decode GEMMs on this GPU, then run all GPU tests and the flagship bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python scripts/bench_gemm.py --tune --m 16 32 48 64 80 96 112 128 \
  --out gpurun_out/gemm_tuning.json > gpurun_out/tune.log 2>&1 || { echo "tune failed"; tail gpurun_out/tune.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [[ $rc != 0 ]] && exit $rc
timeout -k 10 600 python bench.py --steps 3 --warmup 1 --verbose > gpurun_out/bench.log 2>&1
rc=$?; tail -4 gpurun_out/bench.log; exit $rc
