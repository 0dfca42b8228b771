#!/bin/bash
# PMC counters for the prefill attention microbench (kernel-trace + counters only; one pass
# per counter group, each time-boxed; the first failure ends the script).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=$R/gpurun_out/pmc_prefill${PMC_TAG:-}
mkdir -p "$OUT"
cd /tmp
pass() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d "$OUT/$n" -o run --output-format csv \
    -- python3 "$R/scripts/bench_prefill_attn.py" --shapes 1x8192 --qt ${PMC_QT:-32} --iters 2 > "$OUT/$n.log" 2>&1
  local rc=$?; tail -2 "$OUT/$n.log"; return $rc
}
pass p1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU &&
pass p2 SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU &&
pass p3 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_SMEM SQ_WAIT_INST_ANY
