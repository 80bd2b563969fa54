#!/bin/bash
# GPU-box (measurement only): the batch-1 persistent Griffin-Lim loop time and frame-100 phase
# timers for the default library and every variants/lib_*.so, interleaved twice.
set -o pipefail
for k in 1 2; do
  for lib in "" variants/lib_*.so; do
    echo "${lib:-default}: $(env ${lib:+TTS_HIP_LIB=$PWD/$lib} TTS_GL_PHASES=100 timeout -k 10 120 python tools/gl_phases_b1.py 2>&1 | grep -E "PHASES|persistent" | tail -2 | tr '\n' ' ' | sed 's/TTS_GL_PHASES frame 100, us per iteration://')" || exit 1
  done
done
