#!/bin/bash
# GPU-box helper: alternate configs[1] per-sentence timings of the in-tree library and variants/lib_*.so
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  for f in your-voice-tts_amd/libtts_hip.so variants/lib_*.so; do
    r=$(TTS_HIP_LIB=$PWD/$f timeout -k 10 120 python tools/b1_ab.py 2>/dev/null) || { echo "$f failed"; exit 1; }
    echo "$rep $(basename $f) $r"
  done
done
