#!/bin/bash
# GPU-box helper for the batched (configs[2]) path: batched decoder tests, the B=64 bench line and
# its rocprofv3 kernel statistics (gpurun_out/b64_summary.txt).  SKIP_TESTS=1 skips the tests.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_batched.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "batch or overlap or ragged or teacher or config" > gpurun_out/pt_b64.log 2>&1 || { echo batched tests failed; grep -E "FAILED|Error" gpurun_out/pt_b64.log | head; tail -30 gpurun_out/pt_b64.log; exit 1; }
tail -2 gpurun_out/pt_b64.log
fi
timeout -k 10 300 python bench.py --batch 64 --lengths uniform --no-cpu-baseline --no-share > gpurun_out/bench_b64.json 2> gpurun_out/bench_b64.err && python tools/bench_digest.py gpurun_out/bench_b64.json || { tail -20 gpurun_out/bench_b64.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b64 -o run --output-format csv -- python $R/bench.py --batch 64 --lengths uniform --steps 2 --warmup 1 --no-cpu-baseline --no-profile --no-share > $R/gpurun_out/prof_b64_bench.json 2> $R/gpurun_out/prof_b64.err || { echo rocprof failed; tail -20 $R/gpurun_out/prof_b64.err; exit 1; }
python $R/tools/rocprof_summary.py $R/gpurun_out/prof_b64/run_kernel_stats.csv $R/gpurun_out/prof_b64_summary.txt | head -16
