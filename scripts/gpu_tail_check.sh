#!/bin/bash
# Decode tail-split check: its GPU tests, the attention microbench around the 2-per-CU boundary
# (rope vs rope-tail), the engine decode-step profile with EIA_DECODE_TAIL 0 / 4, then the
# endpoint bench.  First failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "${KEXPR:-tail or decode_rope or e2e or engine or canary}" \
  > gpurun_out/tail_tests.log 2>&1 || { tail -40 gpurun_out/tail_tests.log; exit 1; }
tail -2 gpurun_out/tail_tests.log
bash scripts/gpu_attn_batch.sh || exit 1
VALS="${TAILS:-0 4}" bash scripts/gpu_prof_ab.sh EIA_DECODE_TAIL || exit 1
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 400 python -u bench.py > gpurun_out/bench_tail.log 2>&1 || { tail -20 gpurun_out/bench_tail.log; exit 1; }
tail -1 gpurun_out/bench_tail.log
