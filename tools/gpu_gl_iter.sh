#!/bin/bash
# GPU-box helper for persistent Griffin-Lim work: its parity tests, then the phase timers at
# configs[1]'s 222 frames (frame 100) with and without the neighbour wait (TTS_GL_NOWAIT, timing only).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coresidency.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "griffin or persistent or synthesize or sensitivity" > gpurun_out/pt_gl.log 2>&1 || { echo GL tests failed; grep -E "FAILED|Error" gpurun_out/pt_gl.log | head; tail -30 gpurun_out/pt_gl.log; exit 1; }
tail -1 gpurun_out/pt_gl.log
for nw in "" 1; do
  echo "nowait=${nw:-0}"
  env ${nw:+TTS_GL_NOWAIT=1} TTS_GL_PHASES=100 timeout -k 10 120 python tools/gl_phases_b1.py 2>&1 | grep -E "PHASES|persistent" | tail -2 || exit 1
done
