#!/bin/bash
# GPU-box helper for the batch-1 (configs[1]) path: resident decoder / encoder tests, the event
# trace, the bench line and its rocprofv3 kernel statistics (gpurun_out/b1_summary.txt).
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_resident.py tests/test_gpu_coresidency.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "resident or encoder or synthesize or configs1" > gpurun_out/pt_b1.log 2>&1 || { echo b1 tests failed; grep -E "FAILED|Error" gpurun_out/pt_b1.log | head; tail -30 gpurun_out/pt_b1.log; exit 1; }
tail -1 gpurun_out/pt_b1.log
timeout -k 10 200 python tools/resident_trace.py > gpurun_out/trace.json 2>gpurun_out/trace.err || { tail gpurun_out/trace.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/trace.json'))
print('trace us/step', round(d['us_per_step_trace'],3))
for k,v in d['events_rel_step_start_us(min,median,max)'].items(): print(' ', k, v)
print(d['last_cu'])"
timeout -k 10 200 python bench.py --no-cpu-baseline --no-share > gpurun_out/bench_b1.json 2> gpurun_out/bench_b1.err && python tools/bench_digest.py gpurun_out/bench_b1.json || { tail -20 gpurun_out/bench_b1.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
TTS_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b1 -o run --output-format csv -- python $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-profile --no-share > $R/gpurun_out/prof_b1_bench.json 2> $R/gpurun_out/prof_b1.err || { echo rocprof failed; tail -20 $R/gpurun_out/prof_b1.err; exit 1; }
python $R/tools/rocprof_summary.py $R/gpurun_out/prof_b1/run_kernel_stats.csv $R/gpurun_out/prof_b1_summary.txt | head -14
