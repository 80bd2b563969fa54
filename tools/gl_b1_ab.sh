#!/bin/bash
# GPU-box helper: batch-1 Griffin-Lim (222 frames, persistent loop) kernel times per library:
# the in-tree library and variants/lib_*.so, rocprofv3 --stats of tools/gl_phases_b1.py.
set -o pipefail
R=$(pwd)
mkdir -p $R/gpurun_out/glb1
cd /tmp && export TMPDIR=/tmp
for f in $R/your-voice-tts_amd/libtts_hip.so $R/variants/lib_*.so; do
  n=$(basename $f .so)
  TTS_HIP_LIB=$f TTS_COOP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/glb1/$n -o run --output-format csv -- python3 $R/tools/gl_phases_b1.py > $R/gpurun_out/glb1/$n.out 2>&1 || { tail -5 $R/gpurun_out/glb1/$n.out; exit 1; }
  KS=$(ls $R/gpurun_out/glb1/$n/*kernel_stats.csv $R/gpurun_out/glb1/$n/*/*kernel_stats.csv 2>/dev/null | head -1)
  echo "== $n"; python3 $R/tools/rocprof_summary.py $KS /dev/stdout | head -8
  rm -rf $R/gpurun_out/glb1/$n
done
