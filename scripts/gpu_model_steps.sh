#!/bin/bash
# Engine-loop decode-step profile (rocprofv3 kernel trace, last 30 steps) of one model:
# usage: MODEL=mistralai/Mixtral-8x7B-Instruct-v0.1 TAG=mixtral bash scripts/gpu_model_steps.sh
# (BENCH_ARGS: extra bench.py flags, e.g. "--users 35")
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-model}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
( cd /tmp && timeout -k 10 ${LIMIT:-900} rocprofv3 --kernel-trace -d "$OUT" -o run --output-format csv \
    -- python3 "$R/bench.py" --mode engine --model "$MODEL" --steps 1 --warmup 1 ${BENCH_ARGS:-} ) \
    > "gpurun_out/prof_$TAG.log" 2>&1 || { tail -20 "gpurun_out/prof_$TAG.log"; exit 1; }
grep '^{' "gpurun_out/prof_$TAG.log" | tail -1
CSV=$(find "$OUT" -name '*kernel_trace.csv' | head -1)
python3 scripts/analyze_steps.py "$CSV" "$MODEL" 30 > "gpurun_out/steps_$TAG.md" 2>&1 || true
rm -f "$CSV"
head -24 "gpurun_out/steps_$TAG.md"
