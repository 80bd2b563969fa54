#!/bin/bash
# GPU-box helper: rocprofv3 kernel statistics of the batch-1 decoder loop for one attention
# configuration of tools/resident_general_b1.py (resident and multi-launch legs), e.g.
#   CFG=server_fwd_sigmoid_nomask NAME=r05_server bash tools/gpu_general_rocprof.sh
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${NAME:?NAME required}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
TTS_CONFIGS=${CFG:?CFG required} TTS_COOP=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/kt -o run \
  --output-format csv -- python3 $R/tools/resident_general_b1.py > $O/run.log 2> $O/run.err \
  || { echo "kernel trace failed"; tail -20 $O/run.err; exit 1; }
KS=$(ls $O/kt/*kernel_stats.csv $O/kt/*/*kernel_stats.csv 2>/dev/null | head -1)
python3 $R/tools/rocprof_summary.py $KS $O/kernel_stats.txt > /dev/null
head -12 $O/kernel_stats.txt
tail -1 $O/run.log | cut -c1-600
rm -rf $O/kt
