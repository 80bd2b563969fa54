#!/bin/bash
# GPU-box helper: configs[1] A/B of the in-tree library against variants/lib_*.so (tools/b1_ab.sh),
# then the in-tree library's one-sentence timeline (tools/gpu_b1_timeline.sh).  Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
bash tools/b1_ab.sh > gpurun_out/b1_ab.txt 2>&1 || { cat gpurun_out/b1_ab.txt; exit 1; }
cat gpurun_out/b1_ab.txt
bash tools/gpu_b1_timeline.sh > /dev/null || exit 1
cat gpurun_out/b1_timeline2.txt
