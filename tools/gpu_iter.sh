#!/bin/bash
# GPU-box helper for resident-decoder iteration: resident tests, event trace + phases, bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pt_res.log 2>&1 || { echo resident tests failed; tail -40 gpurun_out/pt_res.log; exit 1; }
tail -2 gpurun_out/pt_res.log
timeout -k 10 200 python tools/resident_trace.py > gpurun_out/trace.json 2>gpurun_out/trace.err || { tail gpurun_out/trace.err; exit 1; }
python -c "
import json;d=json.load(open('gpurun_out/trace.json'))
print('trace us/step', round(d['us_per_step_trace'],3))
for k,v in d['events_rel_step_start_us(min,median,max)'].items(): print(' ', k, v)
print(d['last_cu'])"
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err && python tools/bench_digest.py gpurun_out/bench_iter.json
