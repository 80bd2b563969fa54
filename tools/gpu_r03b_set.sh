#!/bin/bash
# GPU-box helper: the late round-3 configs[1] measurement set (bench line, rocprofv3 kernel stats,
# FETCH/WRITE PMC) and the driver-contract default bench line.  Run from the repo root.
set -o pipefail
NAME=r03b_b1 BENCH_ARGS="--no-share" bash tools/gpu_profile.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r03b_default_bench.json 2> gpurun_out/r03b_default_bench.err || { tail -20 gpurun_out/r03b_default_bench.err; exit 1; }
tail -1 gpurun_out/r03b_default_bench.json | cut -c1-400
