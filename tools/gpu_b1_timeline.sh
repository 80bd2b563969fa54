#!/bin/bash
# GPU-box helper: one configs[1] sentence's kernel + copy timeline (pipelined tts_synth_run, as the
# bench's timed loop) -> gpurun_out/b1_timeline.txt.  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
TTS_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $R/gpurun_out/b1tl -o run --output-format csv -- \
  python3 $R/tools/b1_trace.py > $R/gpurun_out/b1tl.log 2>&1 || { echo trace failed; tail -20 $R/gpurun_out/b1tl.log; exit 1; }
cd $R
python3 tools/trace_copies.py gpurun_out/b1tl 12 > gpurun_out/b1_timeline.txt || exit 1
python3 tools/trace_copies.py gpurun_out/b1tl 13 > gpurun_out/b1_timeline2.txt || exit 1
rm -rf gpurun_out/b1tl
cat gpurun_out/b1_timeline.txt
