#!/bin/bash
# Kernel-level profile of the flagship bench: rocprofv3 kernel trace + stats only
# (no PMC here; counters are collected in a separate run).  Engine mode: the endpoint mode
# starts server/client child processes, which must not be exec'd under the profiler.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=$R/gpurun_out/prof_${1:-bench}
mkdir -p "$OUT"
shift || true
cd /tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT" -o run --output-format csv -- \
  python3 "$R/bench.py" --mode engine --steps 1 --warmup 1 "$@" > "$OUT/bench.log" 2>&1
rc=$?
tail -3 "$OUT/bench.log"
find "$OUT" -name '*kernel_stats.csv' -exec head -40 {} \;
exit $rc
