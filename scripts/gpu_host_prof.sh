#!/bin/bash
# Host-side cost of the decode loop: cProfile of the engine-mode bench (the GPU work is
# asynchronous, so the profile is the engine's host path plus its synchronisation points).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
timeout -k 10 400 python -m cProfile -o gpurun_out/host.prof bench.py --mode ${MODE:-engine} \
  --steps 2 --warmup 1 > gpurun_out/host_prof.log 2>&1 || { tail -20 gpurun_out/host_prof.log; exit 1; }
tail -1 gpurun_out/host_prof.log | cut -c1-300
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/host.prof")
with open("gpurun_out/host_prof_top.txt", "w") as f:
    p.stream = f
    p.sort_stats("tottime").print_stats(40)
    p.sort_stats("cumulative").print_stats(70)
PY
