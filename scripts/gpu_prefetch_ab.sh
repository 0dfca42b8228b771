#!/bin/bash
# Infinity Cache prefetch beside decode attention (EIA_MALL_PREFETCH): engine-loop A/B and the
# per-step kernel profile with it on.  First failure ends the script.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
VALS="${VALS:-0 1 0 1}" bash scripts/gpu_ab.sh EIA_MALL_PREFETCH "" 3 || exit 1
VALS="1" bash scripts/gpu_prof_ab.sh EIA_MALL_PREFETCH
