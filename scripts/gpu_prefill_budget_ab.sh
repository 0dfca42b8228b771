#!/bin/bash
# Headline bench with the prefill budget at 8192 tokens / 64 sequences per step (A) and at
# 16384 / 128 (B: the burst's 65 prompts in one step), alternating, two pairs, one box.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for pass in 1 2; do
  timeout -k 10 500 python bench.py --steps 3 --warmup 1 --max-num-batched-tokens 8192 \
    --server-args "--max-num-prefill-seqs 64" > gpurun_out/budget_A_$pass.log 2>&1 || exit 1
  timeout -k 10 500 python bench.py --steps 3 --warmup 1 --max-num-batched-tokens 16384 \
    --server-args "--max-num-prefill-seqs 128" > gpurun_out/budget_B_$pass.log 2>&1 || exit 1
done
for f in gpurun_out/budget_[AB]_*.log; do
  echo "$f $(grep '^{' $f | tail -1 | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ttft_p50_ms"], d["ttft_p90_ms"], d["tpot_p50_ms"], d.get("engine_tok_s"))')"
done
