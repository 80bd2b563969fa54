#!/bin/bash
# GPU-box helper: the full -m gpu suite, then the default bench line and the post-decoder trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_full.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|error" gpurun_out/pt_full.log | head -20; tail -30 gpurun_out/pt_full.log; exit 1; }
tail -2 gpurun_out/pt_full.log
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err && python tools/bench_digest.py gpurun_out/bench_full.json || exit 1
STALL_VARIANTS="base:X=1" bash tools/gpu_stall_ab.sh | sed 's/| scr.*None  //'
