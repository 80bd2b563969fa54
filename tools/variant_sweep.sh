#!/bin/bash
# GPU-box helper: decoder-loop time of the resident decoder per library variant (variants/lib_*.so)
set -o pipefail
mkdir -p gpurun_out
for f in your-voice-tts_amd/libtts_hip.so variants/lib_*.so; do
  TTS_HIP_LIB=$PWD/$f timeout -k 10 120 python tools/resident_phases.py > gpurun_out/ph_$(basename $f).json 2>/dev/null || { echo "$f failed"; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ph_$(basename $f).json')); print('$f', round(d['us_per_step'],2), {k: round(v,2) for k,v in d['phases']['cu0'].items() if v})"
done
