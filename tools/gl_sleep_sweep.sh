#!/bin/bash
# GPU-box helper: persistent Griffin-Lim phases (tools/gl_phases_b1.py) at F = 222 and 342 under
# first-poll delays TTS_GL_FIRST_SLEEP
set -o pipefail
for F in 222 342; do
  for s in 0 4 8 12 16; do
    echo "F=$F sleep=$s"
    GL_F=$F TTS_GL_FIRST_SLEEP=$s TTS_GL_PHASES=100 timeout -k 10 60 python tools/gl_phases_b1.py 2>&1 | grep -v amdgpu.ids || exit 1
    GL_F=$F TTS_GL_FIRST_SLEEP=$s timeout -k 10 60 python tools/gl_phases_b1.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
