#!/bin/bash
# GPU-box helper (measurement only): batch-1 postnet + encoder conv launches -- the per-call time of
# tools/postnet_bench.py, then its rocprofv3 kernel trace: the last postnet + encoder calls' conv
# launches in order with their durations and grids.
set -o pipefail
R=$(pwd); mkdir -p gpurun_out
timeout -k 10 100 python tools/postnet_bench.py 222 100 2>&1 | tail -1 || exit 1
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pn
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/gpurun_out/pn -o run --output-format csv -- python3 $R/tools/postnet_bench.py 222 100 > /dev/null 2>&1 || { echo rocprof failed; exit 1; }
python3 - "$R" <<'PY'
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/gpurun_out/pn/**/*kernel_trace.csv", recursive=True))[0]
rows = list(csv.DictReader(open(f)))
keys = rows[0].keys()
gx = [k for k in keys if k.startswith("Grid")][:1]
seq = [(r["Kernel_Name"].split("(")[0][-40:], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000,
        r[gx[0]] if gx else "") for r in rows]
for s in seq[-40:]: print(s)
PY
rm -rf $R/gpurun_out/pn
