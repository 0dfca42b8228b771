#!/bin/bash
# One measurement session on the GPU box: GPU tests, flagship bench, rocprofv3 kernel stats
# of the bench, decode-GEMM microbenchmark.  Steps are selected by name (default: all);
# each step is time-boxed and the first failure ends the script (no retries).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS=${*:-tests bench prof gemm}
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
    tests) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    ktests) run pytest_k 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$KEXPR" ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 900 python bench.py --steps ${BENCH_STEPS:-3} --warmup 1 --verbose ;;
    prof)
      export TMPDIR=/tmp
      OUT=$R/gpurun_out/prof_bench
      mkdir -p "$OUT"
      ( cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT" -o run \
          --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 1 ) > gpurun_out/prof.log 2>&1
      rc=$?; tail -3 gpurun_out/prof.log; [[ $rc != 0 ]] && { echo "prof rc=$rc"; exit $rc; }
      STATS=$(find "$OUT" -name '*kernel_stats.csv' | head -1)
      python3 scripts/summarize_rocprof.py "$STATS" "rocprofv3 kernel stats: bench.py --steps 1 --warmup 1" 30 \
        > gpurun_out/prof_summary.md 2>&1 || true
      python3 scripts/analyze_trace.py "$OUT" --tail ${TRACE_TAIL:-1.0} > gpurun_out/prof_trace.md 2>&1 || true
      find "$OUT" -name '*kernel_trace.csv' -delete
      head -12 gpurun_out/prof_trace.md ;;
    gemm) run gemm 900 python scripts/bench_gemm.py --sweep --m ${GEMM_M:-65} \
            --shapes qkv_8b o_8b gate_up_8b down_8b lm_head_8b ;;
    attn) run attn 300 python scripts/bench_attn.py ;;
    tune) run tune 1100 python scripts/bench_gemm.py --tune --m ${GEMM_M:-65} \
            --shapes ${GEMM_SHAPES:-qkv_8b o_8b gate_up_8b down_8b lm_head_8b} --out gpurun_out/gemm_tuning.json ;;
    rot)  # staggered K-walk start (EIA_GEMM_ROT) on the tuned configs
      for r in ${ROTS:-0 1 3 7}; do
        EIA_GEMM_ROT=$r run rot_$r 300 python scripts/bench_gemm.py --m ${GEMM_M:-65} \
          --shapes qkv_8b o_8b gate_up_8b down_8b lm_head_8b
      done ;;
    packed) run packed 900 python scripts/bench_gemm.py --packed --sweep --m ${GEMM_M:-65} \
            --shapes ${GEMM_SHAPES:-qkv_8b o_8b gate_up_8b down_8b lm_head_8b} ;;
    sizing) run sizing_8b 1500 python scripts/sizing_sweep.py --model 8b --out gpurun_out/sizing_8b.md ;;
    sizing70) run sizing_70b 1100 python scripts/sizing_sweep.py --model 70b --timeout 600 \
            --cases ${SIZING70_CASES:-chatbot describe translate} --out gpurun_out/sizing_70b_tp1.md ;;
    probe) run probe 300 python scripts/probe_overlap.py ;;
    tei) run tei 900 python scripts/bench_tei.py --window ${TEI_WINDOW:-10} --out gpurun_out/tei.md ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
