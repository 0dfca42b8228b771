set -o pipefail
R=$GRAFT_REPO_ROOT
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p $R/gpurun_out/api
cd /tmp && timeout -k 10 600 rocprofv3 --hip-trace --kernel-trace -d $R/gpurun_out/api -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --output-len 48 > $R/gpurun_out/api.log 2>&1
rc=$?
cd $R && python3 scripts/analyze_api_gaps.py gpurun_out/api --n 3 > gpurun_out/api_gaps.txt 2>&1
find gpurun_out/api -name '*trace.csv' -delete
exit $rc
