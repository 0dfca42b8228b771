#!/bin/bash
# Config #3 readiness on one GPU: the Llama-3.3-70B TP8 rank proxy (catalog
# "llama-70b-tp8-rank") -- decode-step kernel traces at 65 and 35 users, and a full variant
# sweep of its four decode GEMM shapes.  Steps by name (default: all); the first failure ends
# the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS=${*:-artest steps65 steps35 sweep}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -4 "gpurun_out/$name.log"
  if [[ $rc != 0 ]]; then echo "$name rc=$rc"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    artest) run artest 600 python -u -m pytest tests/test_custom_allreduce_gpu.py -m gpu -x -v \
              --timeout 300 --timeout-method thread ;;
    steps65) MODEL=llama-70b-tp8-rank TAG=tp8rank_65 LIMIT=600 bash scripts/gpu_model_steps.sh || exit 1 ;;
    steps35) MODEL=llama-70b-tp8-rank TAG=tp8rank_35 LIMIT=600 BENCH_ARGS="--users 35" \
               bash scripts/gpu_model_steps.sh || exit 1 ;;
    p2|p4) EIA_DECODE_P=${s#p} MODEL=llama-70b-tp8-rank TAG=tp8rank_65_$s LIMIT=600 \
             bash scripts/gpu_model_steps.sh || exit 1 ;;
    sweep) run sweep_tp8 900 python scripts/bench_gemm.py --sweep --all --m ${GEMM_M:-65} \
             --shapes ${GEMM_SHAPES:-qkv_70b_tp8 o_70b_tp8 gate_up_70b_tp8 down_70b_tp8 lm_head_70b_tp8} ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
