#!/bin/bash
# GPU-box helper (diagnostic): per-launch durations around the resident decoder in the pipelined
# configs[1] loop (tools/b1_trace.py) under host-side variants -> gpurun_out/stall_ab.txt
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # label, env assignments..., -- args
  local label=$1; shift
  rm -rf $R/gpurun_out/st_$label
  env "$@" TTS_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/st_$label -o run --output-format csv -- \
    python3 $R/tools/b1_trace.py $ARGS > $R/gpurun_out/st_$label.log 2>&1 || { echo "$label failed"; tail -5 $R/gpurun_out/st_$label.log; exit 1; }
  python3 $R/tools/stall_trace.py $R/gpurun_out/st_$label $label >> $R/gpurun_out/stall_ab.txt || exit 1
  rm -rf $R/gpurun_out/st_$label
}
: > $R/gpurun_out/stall_ab.txt
for v in ${STALL_VARIANTS:-base:X=1 devkarg:HIP_FORCE_DEV_KERNARG=1 hostkarg:HIP_FORCE_DEV_KERNARG=0}; do
  ARGS= run ${v%%:*} ${v#*:} || exit 1
done
cat $R/gpurun_out/stall_ab.txt
