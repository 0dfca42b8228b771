set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out
for d in 2 0 1 3; do
  EIA_MOE_DOWN_CFG=$d timeout -k 10 200 python scripts/bench_moe.py --tokens 65 33 > gpurun_out/moe_d$d.log 2>&1 || { tail -5 gpurun_out/moe_d$d.log; exit 1; }
  echo "down_cfg=$d"; grep -v amdgpu.ids gpurun_out/moe_d$d.log | cut -c1-220
done
for u in 1 0 2; do
  EIA_MOE_UP_CFG=$u timeout -k 10 200 python scripts/bench_moe.py --tokens 65 > gpurun_out/moe_u$u.log 2>&1 || { tail -5 gpurun_out/moe_u$u.log; exit 1; }
  echo "up_cfg=$u"; grep -v amdgpu.ids gpurun_out/moe_u$u.log | cut -c1-220
done
