#!/bin/bash
# Decode attention microbench in engine-like cache states: MALL-hot vs flushed (512 MB read
# sweep before each call) vs flushed with the blocks spread over an engine-sized pool.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for w in ${WAVES:-0 1}; do
  for cfg in "${CFG:-512 16384}"; do
    set -- $cfg
    EIA_DECODE_WAVE=$w timeout -k 10 300 python scripts/bench_attn.py --batch ${BATCHES:-65} \
      --ctx ${CTXS:-192 1024} --p-only 1 2 --fused-sk ${SK:-4} --flush-mb $1 --pool-blocks $2 > gpurun_out/cold_$w.log 2>&1 \
      || { tail -20 gpurun_out/cold_$w.log; exit 1; }
    echo "wave=$w flush=$1 pool=$2: $(grep '"B"' gpurun_out/cold_$w.log | python3 -c 'import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d["B"], d["ctx"], d["all"], "flush_us", d["flush_us"], end=" | ")')"
  done
done
