#!/bin/bash
# GPU-box helper: the round-3 measurement set (bench line, rocprofv3 kernel stats, FETCH/WRITE PMC)
# for configs[1], the configs[2]-shaped batch and configs[4].  Run from the repo root.
set -o pipefail
NAME=r03_b1 BENCH_ARGS="--no-share" bash tools/gpu_profile.sh || exit 1
NAME=r03_b64 BENCH_ARGS="--batch 64 --lengths uniform" bash tools/gpu_profile.sh || exit 1
NAME=r03_gst BENCH_ARGS="--model gst --batch 32" PREFIX=gst_ BENCH_STEPS="--steps 3 --warmup 1" bash tools/gpu_profile.sh || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r03_default_bench.json 2> gpurun_out/r03_default_bench.err || { tail -20 gpurun_out/r03_default_bench.err; exit 1; }
tail -1 gpurun_out/r03_default_bench.json | cut -c1-300
