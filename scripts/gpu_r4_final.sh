#!/bin/bash
# End-of-round evidence on one box: GPU tests, smoke, endpoint bench (burst + closed loop,
# verbose loop phases), endpoint kernel trace (busy fraction / gaps), engine decode-step profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
BENCH_STEPS=5 bash scripts/gpu_session.sh ${*:-tests smoke bench prof} || exit $?
MODEL=meta-llama/Llama-3.1-8B-Instruct TAG=r4_8b bash scripts/gpu_model_steps.sh
