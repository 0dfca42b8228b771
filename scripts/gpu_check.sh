#!/bin/bash
# One GPU session: kernel numerics, smoke, short bench. Each GPU step is time-boxed;
# any failure stops the script (no retries).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEP=${1:-all}
if [[ $STEP == all || $STEP == tests ]]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -5 gpurun_out/pytest_gpu.log; [[ $rc != 0 ]] && { echo "pytest rc=$rc"; exit $rc; }
fi
if [[ $STEP == all || $STEP == smoke ]]; then
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
  rc=$?; tail -3 gpurun_out/smoke.log; [[ $rc != 0 ]] && { echo "smoke rc=$rc"; exit $rc; }
fi
if [[ $STEP == all || $STEP == bench ]]; then
  timeout -k 10 900 python bench.py --steps ${BENCH_STEPS:-2} --warmup 1 --verbose > gpurun_out/bench.log 2>&1
  rc=$?; tail -4 gpurun_out/bench.log; [[ $rc != 0 ]] && { echo "bench rc=$rc"; exit $rc; }
fi
exit 0
