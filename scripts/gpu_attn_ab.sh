#!/bin/bash
# Decode attention A/B (4-wave form vs one-wave form): phase trace, cold microbench with the
# fused RoPE form, GPU kernel tests, engine decode-step profile.  First failure ends it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for w in ${WAVES:-0 1}; do
  echo "== EIA_DECODE_WAVE=$w"
  EIA_DECODE_WAVE=$w timeout -k 10 120 python scripts/attn_trace.py --ctx ${TRACE_CTX:-192} || exit 1
done
WAVES="${WAVES:-0 1}" CTXS="${CTXS:-192 1024 4096}" bash scripts/gpu_attn_cold.sh || exit 1
KEXPR="${KEXPR:-decode or rope or attention or engine or e2e or canary}" WAVES="${WAVES:-0 1}" \
  bash scripts/gpu_decode_check.sh
