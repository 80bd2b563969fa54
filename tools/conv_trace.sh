#!/bin/bash
# GPU-box helper (diagnostic): per-dispatch durations of the conv kernels in one configs[2] bench
# step (kernel trace CSV summarised in order of dispatch).  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/ct -o run --output-format csv -- \
  python3 $R/bench.py --batch 64 --lengths uniform --steps 1 --warmup 0 --no-cpu-baseline --no-profile > $R/gpurun_out/ct.json 2> $R/gpurun_out/ct.err \
  || { echo "trace failed"; tail -5 $R/gpurun_out/ct.err; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob
f = sorted(glob.glob('gpurun_out/ct/**/*kernel_trace.csv', recursive=True))[0]
rows = [r for r in csv.DictReader(open(f)) if 'conv' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for r in rows:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    print(f"{d:9.1f} us  grid {r.get('Grid_Size_X', r.get('Grid_Size', '?'))}  {r['Kernel_Name'][:70]}")
PY
rm -rf gpurun_out/ct
