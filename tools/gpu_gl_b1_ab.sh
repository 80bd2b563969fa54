#!/bin/bash
# GPU-box helper: batch-1 persistent Griffin-Lim phase timers (tools/gl_phases_b1.py) and configs[1]
# per-sentence times (tools/b1_ab.py) for the in-tree library and each variants/lib_*.so.
set -o pipefail
for f in your-voice-tts_amd/libtts_hip.so variants/lib_*.so; do
  echo "== $f"
  TTS_HIP_LIB=$PWD/$f TTS_GL_PHASES=100 timeout -k 10 120 python tools/gl_phases_b1.py 2>&1 | grep -E "PHASES|persistent" | tail -2 || exit 1
  TTS_HIP_LIB=$PWD/$f timeout -k 10 120 python tools/b1_ab.py 2>/dev/null || exit 1
done
