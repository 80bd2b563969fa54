#!/bin/bash
# GPU-box helper: Griffin-Lim A/B of the in-tree library against variants/lib_*.so: configs[2]
# (B=64) and configs[4] (GST B=32) per-iteration kernel times (tts_gl_profile) and bench values.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for f in your-voice-tts_amd/libtts_hip.so variants/lib_*.so; do
    n=$(basename $f .so)
    TTS_HIP_LIB=$PWD/$f timeout -k 10 200 python bench.py --batch 64 --lengths uniform --steps 3 --warmup 1 --no-cpu-baseline --no-share > gpurun_out/glab_${n}.json 2> gpurun_out/glab_${n}.err || { tail -20 gpurun_out/glab_${n}.err; exit 1; }
    TTS_HIP_LIB=$PWD/$f timeout -k 10 200 python bench.py --model gst --batch 32 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/glabg_${n}.json 2> gpurun_out/glabg_${n}.err || { tail -20 gpurun_out/glabg_${n}.err; exit 1; }
    python - <<PY
import json
ld=lambda p:[json.loads(l) for l in open(p) if l.startswith('{')][0]
d=ld('gpurun_out/glab_${n}.json'); e=ld('gpurun_out/glabg_${n}.json')
k=d['kernels_rank0']; kg=e['kernels_rank0']
print('$rep $n', 'b64', round(d['value']), round(d['stages_rank0']['griffin_lim_ms'],2), 'gl_iter_ms', round(k['gl_iter']['mean_ms']*1e3,1),
      '| gst', round(e['value']), round(e['stages_rank0']['griffin_lim_ms'],2), 'gl_iter_ms', round(kg['gl_iter']['mean_ms']*1e3,1))
PY
  done
done
