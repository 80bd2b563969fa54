#!/bin/bash
# GPU-box helper (round 3 state check): full GPU suite + bench + kernel stats, then the batch-1
# Griffin-Lim phase timers.  Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_test_bench.sh || exit 1
TTS_GL_PHASES=100 timeout -k 10 120 python tools/gl_phases_b1.py > gpurun_out/gl_phases.txt 2>&1 || { echo gl phases failed; tail -20 gpurun_out/gl_phases.txt; exit 1; }
tail -5 gpurun_out/gl_phases.txt
