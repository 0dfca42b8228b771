#!/bin/bash
# Does the 8B QKV's split-K cost the decode attention more than it saves the GEMM?  Sweep the
# QKV at 65 / 72 rows (plain and workgroup-packed, every split), force the best whole-K (sk 1)
# pick into a copy of the table, and trace the engine's decode steps with each table.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python scripts/bench_gemm.py --sweep --all --wgpack --m 65 72 --shapes qkv_8b \
  > gpurun_out/qkv8b_sweep.log 2>&1 || exit 1
python - <<'PY' || exit 1
import json
rows = [json.loads(l) for l in open("gpurun_out/qkv8b_sweep.log") if l.startswith("{")]
tot = {}
for r in rows:
    for t, c, s in r["all"]:
        if s == 1:
            tot.setdefault(c, []).append(t)
best = min((sum(v), c) for c, v in tot.items() if len(v) == len(rows))
print("best sk=1 QKV cfg", best)
t = json.load(open("enterprise_inference_amd/ops/gemm_tuning.json"))
for mt in (4, 5, 6):
    key = f"{mt},6144,4096,0"
    if best[1] & 1024:
        t["wg_entries"][key] = [best[1], 1]
    else:
        t["wg_entries"].pop(key, None)
        t["entries"][key] = [best[1], 1]
json.dump(t, open("gpurun_out/table_qkv_sk1.json", "w"), indent=0, sort_keys=True)
PY
MODEL=llama-8b TAG=8b_qkvsk4 LIMIT=400 bash scripts/gpu_model_steps.sh > /dev/null || exit 1
EIA_GEMM_TUNING=gpurun_out/table_qkv_sk1.json MODEL=llama-8b TAG=8b_qkvsk1 LIMIT=400 \
  bash scripts/gpu_model_steps.sh > /dev/null || exit 1
for t in 8b_qkvsk4 8b_qkvsk1; do head -3 gpurun_out/steps_$t.md | tail -1; grep -E "paged_decode|12288x|6144|<5, 2, 3" gpurun_out/steps_$t.md | head -6; done
