set -o pipefail
mkdir -p gpurun_out/prof_burst
export TMPDIR=/tmp
R=$PWD
( cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_burst -o run --output-format csv -- python3 $R/scripts/burst_timeline.py --model llama-8b --out $R/gpurun_out/burst_8b_prof.md ) > gpurun_out/burst_prof.log 2>&1
CSV=$(find gpurun_out/prof_burst -name '*kernel_trace.csv' | head -1)
python3 scripts/trace_gaps.py "$CSV" --after-gap-ms 50 --window-ms 110 > gpurun_out/burst_gaps.txt
rm -f "$CSV"
