#!/bin/bash
# Fused decode attention vs batch size around the 2-workgroups-per-CU boundary (B 64 = 512
# workgroups, 65 = 520, 72 = 576), cold Infinity Cache, P 1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
for B in ${BATCHES:-64 65 72}; do
  timeout -k 10 100 python scripts/bench_attn.py --batch $B --ctx ${CTXS:-192 256} --p-only 1 \
    --fused-sk 4 --tail-parts ${TAILP:-}  --flush-mb 512 --pool-blocks 16384 2>/dev/null > gpurun_out/attn_b$B.log || exit 1
  python3 - "$B" <<'PY'
import json, sys
for l in open(f"gpurun_out/attn_b{sys.argv[1]}.log"):
    if l.startswith("{"):
        d = json.loads(l)
        print(d["B"], d["ctx"], d["all"])
PY
done
