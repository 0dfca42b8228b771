#!/bin/bash
# Endpoint headline with the intake coalescing gap at 2 ms (default) and 6 ms.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for g in 2 6 2 6; do
  EIA_INTAKE_GAP_MS=$g timeout -k 10 400 python bench.py --steps 5 --warmup 1 --verbose --closed-loop-s 0 > gpurun_out/intake_g$g.log 2>&1 || exit 1
  echo "gap=$g $(grep -o 'round [0-9]: .*' gpurun_out/intake_g$g.log | tr '\n' ' ' | cut -c1-400)"
  echo "   $(grep -o 'loop_times.*' gpurun_out/intake_g$g.log)"
  echo "   $(tail -1 gpurun_out/intake_g$g.log | grep -o '"value": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"tpot_p50_ms": [0-9.]*' | tr '\n' ' ')"
done
