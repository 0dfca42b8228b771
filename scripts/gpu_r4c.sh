#!/bin/bash
# Host loop phases of the engine core under the endpoint bench (where the step-boundary idle
# comes from), and the engine-loop reference.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --verbose --closed-loop-s 8 > gpurun_out/bench_ep.log 2>&1
rc=$?; grep -v "^\[replica" gpurun_out/bench_ep.log | tail -3; grep "ms/step" gpurun_out/bench_ep.log; [[ $rc != 0 ]] && exit $rc
timeout -k 10 600 python bench.py --mode engine --steps 5 --warmup 2 --verbose > gpurun_out/bench_eng.log 2>&1
rc=$?; tail -3 gpurun_out/bench_eng.log; exit $rc
