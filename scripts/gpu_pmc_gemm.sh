#!/bin/bash
# PMC counters for the decode GEMM microbench (kernel-trace + counters only; no sys/hip trace).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=$R/gpurun_out/pmc_gemm
mkdir -p "$OUT"
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS FETCH_SIZE \
  -d "$OUT" -o run --output-format csv -- python3 "$R/scripts/bench_gemm.py" --shapes gate_up_8b lm_head_8b --m 16 80 --iters 5 \
  > "$OUT/log.txt" 2>&1
rc=$?; tail -5 "$OUT/log.txt"; exit $rc
