#!/bin/bash
# GPU-box helper: batched bench lines -- configs[2] shape (Tacotron2 batch 64, uniform LJSpeech-like
# lengths) and configs[4] (TacotronGST batch 32) -- each followed by a rocprofv3 kernel summary.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --batch 64 --lengths uniform --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_b64.json 2> gpurun_out/bench_b64.err || { echo b64 bench failed; tail -30 gpurun_out/bench_b64.err; exit 1; }
cat gpurun_out/bench_b64.json
timeout -k 10 300 python bench.py --model gst --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_gst.json 2> gpurun_out/bench_gst.err || { echo gst bench failed; tail -30 gpurun_out/bench_gst.err; exit 1; }
cat gpurun_out/bench_gst.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b64 -o run --output-format csv -- python $R/bench.py --batch 64 --lengths uniform --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $R/gpurun_out/prof_b64_bench.json 2> $R/gpurun_out/prof_b64.err || { echo rocprof failed; tail -20 $R/gpurun_out/prof_b64.err; exit 1; }
python $R/tools/rocprof_summary.py $R/gpurun_out/prof_b64/run_kernel_stats.csv $R/gpurun_out/prof_b64_summary.txt | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_gst -o run --output-format csv -- python $R/bench.py --model gst --batch 32 --steps 2 --warmup 1 --no-cpu-baseline --no-profile > $R/gpurun_out/prof_gst_bench.json 2> $R/gpurun_out/prof_gst.err || { echo rocprof failed; tail -20 $R/gpurun_out/prof_gst.err; exit 1; }
python $R/tools/rocprof_summary.py $R/gpurun_out/prof_gst/run_kernel_stats.csv $R/gpurun_out/prof_gst_summary.txt | head -12
