#!/bin/bash
# Host HIP API calls around the GPU idle gaps of the decode loop (rocprofv3 hip + kernel +
# memory-copy traces, no counters), engine mode by default (MODE=endpoint for the server).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p $R/gpurun_out/api
cd /tmp && timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -d $R/gpurun_out/api -o run \
  --output-format csv -- python3 $R/bench.py --mode ${MODE:-engine} --steps 1 --warmup 1 --output-len 48 --verbose \
  > $R/gpurun_out/api.log 2>&1
rc=$?
cd $R && python3 scripts/analyze_api_gaps.py gpurun_out/api --n ${NGAPS:-4} --lookback-ms ${LOOKBACK_MS:-6} \
  > gpurun_out/api_gaps.txt 2>&1
find gpurun_out/api -name '*trace.csv' -delete
exit $rc
