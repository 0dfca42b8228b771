#!/bin/bash
# Dense decode GEMMs: staggered K walk on the split-K table picks too (EIA_GEMM_ROT=3) vs the
# default (single-split only), table picks timed at the headline / 70B rows.
set -o pipefail
mkdir -p gpurun_out
for r in -1 3 -1 3; do
  if [ "$r" = "-1" ]; then unset EIA_GEMM_ROT; else export EIA_GEMM_ROT=$r; fi
  timeout -k 10 300 python scripts/bench_gemm.py --m 35 65 --shapes qkv_8b o_8b down_8b o_70b down_70b --iters 30 > gpurun_out/rot_sk_$r.log 2>&1 || exit 1
  echo "rot=$r"; grep '^{' gpurun_out/rot_sk_$r.log | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(' ', d['shape'], d['M'], d.get('cfg'), d.get('sk'), d.get('ours_us'))"
done
