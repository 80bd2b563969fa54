#!/bin/bash
# GPU-box helper (diagnostic): SQ instruction / wait counters of the persistent Griffin-Lim over the
# pipelined configs[1] loop -> gpurun_out/gl_sq.txt (counter list -> gpurun_out/counters.txt)
set -o pipefail
R=$(pwd); mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > $R/gpurun_out/counters.txt 2>&1 || true
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
         "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"; do
  rm -rf $R/gpurun_out/glsq
  TTS_COOP=0 timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/glsq -o run --output-format csv -- \
    python3 $R/tools/b1_trace.py > $R/gpurun_out/glsq.log 2>&1 || { echo "pmc failed: $P"; tail -5 $R/gpurun_out/glsq.log; exit 1; }
  python3 - "$R" <<'PY' >> $R/gpurun_out/gl_sq.txt
import csv, glob, sys, collections
R = sys.argv[1]
cc = glob.glob(R + "/gpurun_out/glsq/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(cc)):
    if "gl_persistent" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    v = sorted(v)[len(v) // 2]
    print(f"{k:28s} {v:16.0f}")
PY
done
rm -rf $R/gpurun_out/glsq
cat $R/gpurun_out/gl_sq.txt
