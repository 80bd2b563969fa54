#!/bin/bash
# GPU-box helper (diagnostic): GRBM_COUNT / GRBM_GUI_ACTIVE per dispatch over tools/b1_trace.py, to
# tell a clock drop from a longer kernel -> gpurun_out/clock_pmc.txt.  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
TTS_COOP=0 timeout -s KILL 120 rocprofv3 --pmc GRBM_COUNT GRBM_GUI_ACTIVE --kernel-trace -d $R/gpurun_out/clk -o run \
  --output-format csv -- python3 $R/tools/b1_trace.py > $R/gpurun_out/clk.log 2>&1 || { echo "pmc failed"; tail -20 $R/gpurun_out/clk.log; exit 1; }
cd $R
python3 - <<'PY' > gpurun_out/clock_pmc.txt
import csv, glob, collections
cc = glob.glob("gpurun_out/clk/**/*counter_collection.csv", recursive=True)[0]
kt = glob.glob("gpurun_out/clk/**/*kernel_trace.csv", recursive=True)
rows = list(csv.DictReader(open(cc)))
print(list(rows[0].keys()))
per = collections.OrderedDict()
for r in rows:
    key = (r.get("Dispatch_Id") or r.get("Correlation_Id"), r["Kernel_Name"][:50])
    per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    for k in ("Start_Timestamp", "End_Timestamp"):
        if k in r: per[key][k] = int(r[k])
items = list(per.items())[-60:]
for (d, n), v in items:
    dur = (v.get("End_Timestamp", 0) - v.get("Start_Timestamp", 0)) / 1e3
    print(f"{n:50s} dur {dur:9.1f} us  GRBM_COUNT {v.get('GRBM_COUNT', 0):10.0f}  GUI_ACTIVE {v.get('GRBM_GUI_ACTIVE', 0):10.0f}")
PY
rm -rf gpurun_out/clk
cat gpurun_out/clock_pmc.txt | tail -45
