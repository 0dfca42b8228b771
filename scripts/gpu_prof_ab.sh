#!/bin/bash
# rocprofv3 kernel trace of the engine-mode bench under VAR=v for each v, summarised per decode
# step by scripts/analyze_steps.py (last 30 steps).  usage: VALS="0 1" bash scripts/gpu_prof_ab.sh VAR
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
VAR=$1
for v in ${VALS:-0 1}; do
  OUT=$R/gpurun_out/prof_${VAR}_$v
  mkdir -p "$OUT"
  ( cd /tmp && export "$VAR=$v" && timeout -k 10 600 rocprofv3 --kernel-trace -d "$OUT" -o run \
      --output-format csv -- python3 "$R/bench.py" --mode engine --steps 1 --warmup 1 ) \
      > "gpurun_out/prof_${VAR}_$v.log" 2>&1 || { tail -20 "gpurun_out/prof_${VAR}_$v.log"; exit 1; }
  CSV=$(find "$OUT" -name '*kernel_trace.csv' | head -1)
  python3 scripts/analyze_steps.py "$CSV" "$VAR=$v" 30 > "gpurun_out/steps_${VAR}_$v.md" 2>&1 || true
  rm -f "$CSV"
  head -14 "gpurun_out/steps_${VAR}_$v.md"
done
