set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k decode_rope_fused -x -q --timeout 120 --timeout-method thread > gpurun_out/t_rope.log 2>&1 || { tail -30 gpurun_out/t_rope.log; exit 1; }
tail -2 gpurun_out/t_rope.log
timeout -k 10 600 python -u scripts/bench_gemm.py --tune --m 33 40 48 65 72 --shapes qkv_405b_tp8 --out gpurun_out/gemm_tuning.json > gpurun_out/tune_qkv405.log 2>&1 || exit 1
timeout -k 10 600 python -u scripts/bench_gemm.py --tune --wgpack --m 33 40 48 65 72 --shapes qkv_405b_tp8 --out gpurun_out/gemm_tuning.json > gpurun_out/tune_qkv405_wg.log 2>&1 || exit 1
export EIA_WG_PACK_KV_KEEP=0.30
bash scripts/gpu_catalog.sh rank405 steps405
