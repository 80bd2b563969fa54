#!/bin/bash
# GPU-box helper (diagnostic): per-dispatch SQ/GRBM counters over the pipelined configs[1] loop, to
# tell whether a slow post-decoder launch's waves did more work or started late -> gpurun_out/stall_pmc.txt
set -o pipefail
R=$(pwd); mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
TTS_COOP=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT \
  --kernel-trace -d $R/gpurun_out/spmc -o run --output-format csv -- python3 $R/tools/b1_trace.py > $R/gpurun_out/spmc.log 2>&1 || { echo "pmc failed"; tail -20 $R/gpurun_out/spmc.log; exit 1; }
cd $R
python3 - <<'PY' > gpurun_out/stall_pmc.txt
import csv, glob, collections
cc = glob.glob("gpurun_out/spmc/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(cc)))
per = collections.OrderedDict()
for r in rows:
    key = (int(r.get("Dispatch_Id") or r.get("Correlation_Id")), r["Kernel_Name"].replace("void ", "").replace("tts::", "").replace("(anonymous namespace)::", "").split("(")[0][:28])
    per.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    for k in ("Start_Timestamp", "End_Timestamp"):
        if k in r: per[key][k] = int(r[k])
items = list(per.items())[-45:]
cols = ["SQ_WAVES", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE", "GRBM_COUNT"]
print(f"{'kernel':28s} {'dur_us':>8s} " + " ".join(f"{c[3:15]:>12s}" for c in cols))
for (d, n), v in items:
    dur = (v.get("End_Timestamp", 0) - v.get("Start_Timestamp", 0)) / 1e3
    print(f"{n:28s} {dur:8.1f} " + " ".join(f"{v.get(c, 0):12.0f}" for c in cols))
PY
rm -rf gpurun_out/spmc
cat gpurun_out/stall_pmc.txt
