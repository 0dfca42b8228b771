#!/bin/bash
# Config #4 (Mixtral-8x7B, one GPU, 65 users, 128/128) through the OpenAI endpoint: burst rounds
# plus the closed-loop window; the engine-loop number beside it for the step time.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
M=mistralai/Mixtral-8x7B-Instruct-v0.1
timeout -k 10 900 python bench.py --model $M --steps 3 --warmup 1 --verbose > gpurun_out/mixtral_ep.log 2>&1
rc=$?; tail -3 gpurun_out/mixtral_ep.log | cut -c1-1500; [[ $rc != 0 ]] && exit $rc
timeout -k 10 600 python bench.py --model $M --mode engine --steps 3 --warmup 1 > gpurun_out/mixtral_eng.log 2>&1
rc=$?; tail -1 gpurun_out/mixtral_eng.log | cut -c1-600; exit $rc
