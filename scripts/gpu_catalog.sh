#!/bin/bash
# Rest-of-catalog measurements on one MI355X: decode-GEMM tables for Llama-4-Scout's dense
# shapes, endpoint chatbot rows (65 users, 128/128) for Llama-4-Scout-17B-16E and Mistral-7B,
# TEI embedding / rerank throughput, and the TP8-rank GEMM sweep.  Steps by name; the first
# failure ends the script (no retries).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
STEPS=${*:-tune_scout scout mistral tei}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  tail -3 "gpurun_out/$name.log" | cut -c1-400
  if [[ $rc != 0 ]]; then echo "$name rc=$rc"; exit $rc; fi
}
for s in $STEPS; do
  case $s in
    tune_scout) run tune_scout 900 python scripts/bench_gemm.py --tune --m ${SCOUT_M:-33 40 48 65 72 80} \
                  --shapes qkv_scout o_scout shared_gate_up_scout shared_down_scout lm_head_scout \
                  --out gpurun_out/gemm_tuning.json ;;
    scout) run endpoint_scout 1100 python bench.py --model llama-4-scout-17b --steps 2 --warmup 1 \
             --extras off --verbose ;;
    mistral) run endpoint_mistral 600 python bench.py --model mistral-7b --steps 3 --warmup 1 \
               --verbose ;;
    codellama) run endpoint_codellama 900 python bench.py --model codellama-34b --steps 2 \
                 --warmup 1 --verbose ;;
    dsqwen) run endpoint_dsqwen 900 python bench.py --model deepseek-r1-distill-qwen-32b --steps 2 \
              --warmup 1 --verbose ;;
    dsllama) run endpoint_dsllama 600 python bench.py --model deepseek-r1-distill-llama8b --steps 3 \
               --warmup 1 --verbose ;;
    tei) run tei 900 python scripts/bench_tei.py --window ${TEI_WINDOW:-10} --out gpurun_out/tei.md ;;
    tune_tp8) run tune_tp8 900 python scripts/bench_gemm.py --tune --m ${TP8_M:-33 40 48 65 72 80} \
                --shapes qkv_70b_tp8 o_70b_tp8 gate_up_70b_tp8 down_70b_tp8 \
                --out gpurun_out/gemm_tuning.json ;;
    tune_tp8_wg) run tune_tp8_wg 900 python scripts/bench_gemm.py --tune --wgpack \
                   --m ${TP8_M:-33 40 48 65 72 80} \
                   --shapes qkv_70b_tp8 o_70b_tp8 gate_up_70b_tp8 down_70b_tp8 \
                   --out gpurun_out/gemm_tuning.json ;;
    retune) cp enterprise_inference_amd/ops/gemm_tuning.json gpurun_out/table_before.json
            run retune 900 python scripts/bench_gemm.py --tune --m ${RT_M:-33 40 48 65 72 80} \
              --shapes ${RT_SHAPES:-qkv_8b o_8b down_8b qkv_70b_tp8 o_70b_tp8 down_70b_tp8} \
              --out gpurun_out/gemm_tuning.json
            run retune_wg 900 python scripts/bench_gemm.py --tune --wgpack --m ${RT_M:-33 40 48 65 72 80} \
              --shapes ${RT_SHAPES:-qkv_8b o_8b down_8b qkv_70b_tp8 o_70b_tp8 down_70b_tp8} \
              --out gpurun_out/gemm_tuning.json
            cp enterprise_inference_amd/ops/gemm_tuning.json gpurun_out/table_after.json ;;
    abtable)   # engine loop, headline config, table before / after the re-tune, alternating
      for t in before after before after; do
        EIA_GEMM_TUNING=$R/gpurun_out/table_$t.json timeout -k 10 600 python bench.py --mode engine \
          --steps 3 --warmup 1 > gpurun_out/abtable_$t.log 2>&1 || { tail -20 gpurun_out/abtable_$t.log; exit 1; }
        echo "table=$t $(grep -o '"value": [0-9.]*\|"tpot_p50_ms": [0-9.]*' gpurun_out/abtable_$t.log | tr '\n' ' ')"
      done ;;
    tune_405) run tune_405 900 python scripts/bench_gemm.py --tune --m ${T405_M:-33 40 48 65 72} \
                --shapes qkv_405b_tp8 o_405b_tp8 gate_up_405b_tp8 down_405b_tp8 lm_head_405b_tp8 \
                --out gpurun_out/gemm_tuning.json
              run tune_405_wg 900 env EIA_GEMM_TUNING=gpurun_out/gemm_tuning.json \
                python scripts/bench_gemm.py --tune --wgpack --m ${T405_M:-33 40 48 65 72} \
                --shapes qkv_405b_tp8 o_405b_tp8 gate_up_405b_tp8 down_405b_tp8 lm_head_405b_tp8 \
                --out gpurun_out/gemm_tuning.json ;;
    # the 405B TP8 rank proxy (~101 GB) at the reference's 405B chatbot row (35 users, 128/128)
    rank405) run engine_405_rank 900 env EIA_GEMM_TUNING=${T405_TABLE:-enterprise_inference_amd/ops/gemm_tuning.json} \
               python bench.py --mode engine --model llama-405b-tp8-rank --users 35 --steps 2 \
               --warmup 1 --verbose ;;
    steps405) EIA_GEMM_TUNING=${T405_TABLE:-enterprise_inference_amd/ops/gemm_tuning.json} \
                MODEL=llama-405b-tp8-rank TAG=405b_rank BENCH_ARGS="--users 35" LIMIT=900 \
                bash scripts/gpu_model_steps.sh > gpurun_out/steps405.log 2>&1 || exit 1 ;;
    sweep_tp8) run sweep_tp8 900 python scripts/bench_gemm.py --sweep --all --m ${GEMM_M:-65} \
                 --shapes qkv_70b_tp8 o_70b_tp8 gate_up_70b_tp8 down_70b_tp8 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
