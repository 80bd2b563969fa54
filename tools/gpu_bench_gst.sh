#!/bin/bash
# GPU-box helper: configs[4] (TacotronGST, batch 32) bench line + rocprofv3 kernel summary.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 600 python bench.py --model gst --batch 32 --steps 3 --warmup 1 ${BENCH_ARGS} > gpurun_out/bench_gst.json 2> gpurun_out/bench_gst.err || { echo bench failed; tail -30 gpurun_out/bench_gst.err; exit 1; }
cat gpurun_out/bench_gst.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gst -o run --output-format csv -- python $R/bench.py --model gst --batch 32 --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/prof_gst_bench.json 2> $R/gpurun_out/prof_gst.err || { echo rocprof failed; tail -20 $R/gpurun_out/prof_gst.err; exit 1; }
python $R/tools/rocprof_summary.py $R/gpurun_out/prof_gst/run_kernel_stats.csv $R/gpurun_out/prof_gst_summary.txt | head -30
