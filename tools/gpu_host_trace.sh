#!/bin/bash
# GPU-box helper (diagnostic): host API + kernel timeline of one pipelined configs[1] sentence
set -o pipefail
R=$(pwd); mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
TTS_COOP=0 timeout -k 10 120 rocprofv3 --hip-trace --kernel-trace -d $R/gpurun_out/ht -o run --output-format csv -- \
  python3 $R/tools/b1_trace.py > $R/gpurun_out/ht.log 2>&1 || { tail -5 $R/gpurun_out/ht.log; exit 1; }
python3 $R/tools/host_trace.py $R/gpurun_out/ht 12 > $R/gpurun_out/host_trace.txt || exit 1
rm -rf $R/gpurun_out/ht
wc -l $R/gpurun_out/host_trace.txt
