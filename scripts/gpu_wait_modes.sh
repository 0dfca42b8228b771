#!/bin/bash
# Compare host wait strategies for in-flight sampled tokens (overlapped scheduling).
set -o pipefail
mkdir -p gpurun_out
for m in event blocking spin yield; do
  EIA_TOKEN_WAIT=$m timeout -k 10 300 python bench.py --steps 2 --warmup 1 --verbose > gpurun_out/wait_$m.log 2>&1 || { echo "$m failed"; tail -5 gpurun_out/wait_$m.log; exit 1; }
  echo "$m: $(grep -o '"value": [0-9.]*' gpurun_out/wait_$m.log) $(grep 'host ms' gpurun_out/wait_$m.log)"
done
