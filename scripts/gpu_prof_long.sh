set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R; mkdir -p gpurun_out/prof_long; export TMPDIR=/tmp
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_long -o run --output-format csv -- python3 $R/bench.py --steps 1 --warmup 1 --users 16 --input-len 8192 --output-len 16 --max-num-batched-tokens 8192 ) > gpurun_out/prof_long.log 2>&1
rc=$?; tail -3 gpurun_out/prof_long.log; [[ $rc != 0 ]] && exit $rc
STATS=$(find gpurun_out/prof_long -name '*kernel_stats.csv' | head -1)
python3 scripts/summarize_rocprof.py "$STATS" "rocprofv3 kernel stats: 8B, 16 users x 8192 in / 16 out" 25 > gpurun_out/prof_long_summary.md
find gpurun_out/prof_long -name '*kernel_trace.csv' -delete
cat gpurun_out/prof_long_summary.md
