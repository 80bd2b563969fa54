#!/bin/bash
# GPU-box helper (measurement only): persistent Griffin-Lim phase timers at configs[1]'s 222 frames,
# with the neighbour wait (default) and with TTS_GL_NOWAIT=1 (one gather sweep, tags unchecked).
set -o pipefail
for f in 100 3 50; do
  for nw in "" 1; do
    echo "frame $f nowait=${nw:-0}"
    env ${nw:+TTS_GL_NOWAIT=1} TTS_GL_PHASES=$f timeout -k 10 120 python tools/gl_phases_b1.py 2>&1 | grep -E "PHASES|persistent" | tail -2 || exit 1
  done
done
