#!/bin/bash
# GPU-box helper: parity tests, then bench + rocprofv3 kernel-trace summary.  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 || { echo tests failed; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo bench failed; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS} > $R/gpurun_out/prof_bench.json 2> $R/gpurun_out/prof.err || { echo rocprof failed; tail -20 $R/gpurun_out/prof.err; exit 1; }
python $R/tools/rocprof_summary.py $R/gpurun_out/prof/run_kernel_stats.csv $R/gpurun_out/prof_summary.txt | head -16
