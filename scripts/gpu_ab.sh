#!/bin/bash
# A/B of an env switch on the flagship engine loop: GPU tests selected by -k, then
# bench.py --mode engine with VAR=0 and VAR=1 (each time-boxed; first failure ends the script).
#   usage: bash scripts/gpu_ab.sh VAR "pytest -k expr" [steps]   (VALS, MODE, BENCH_ARGS env)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VAR=$1; KEXPR=$2; STEPS=${3:-3}
if [[ -n "$KEXPR" ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "$KEXPR" > gpurun_out/ab_tests.log 2>&1 || { tail -30 gpurun_out/ab_tests.log; exit 1; }
  tail -2 gpurun_out/ab_tests.log
fi
for v in ${VALS:-0 1 0 1}; do
  env "$VAR=$v" timeout -k 10 600 python bench.py --mode ${MODE:-engine} --steps "$STEPS" --warmup 1 ${BENCH_ARGS:-} \
    > "gpurun_out/ab_${VAR}_$v.log" 2>&1 || { tail -20 "gpurun_out/ab_${VAR}_$v.log"; exit 1; }
  echo "$VAR=$v $(grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' gpurun_out/ab_${VAR}_$v.log | tr '\n' ' ')"
done
