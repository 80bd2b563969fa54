#!/bin/bash
# GPU-box helper: rocprofv3 kernel traces of tools/b1_trace.py for each "name|ENV=...|lib" line of
# $CASES (default: the in-tree library and each variants/lib_*.so), then per-kernel mean durations
# side by side (tools/b1_kernel_ab.py).  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
if [ -z "$CASES" ]; then
  CASES=$(for f in your-voice-tts_amd/libtts_hip.so variants/lib_*.so; do [ -f "$f" ] && echo "$(basename $f .so)|X=1|$f"; done)
fi
cd /tmp && export TMPDIR=/tmp
dirs=""
while IFS='|' read -r n envs f; do
  [ -z "$n" ] && continue
  env $envs TTS_HIP_LIB=$R/$f TTS_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace -d $R/gpurun_out/kab_$n -o run --output-format csv -- \
    python3 $R/tools/b1_trace.py > $R/gpurun_out/kab_$n.log 2>&1 || { echo "trace $n failed"; tail -20 $R/gpurun_out/kab_$n.log; exit 1; }
  dirs="$dirs $R/gpurun_out/kab_$n"
done <<< "$CASES"
cd $R
python3 tools/b1_kernel_ab.py $dirs | tee gpurun_out/b1_kernel_ab.txt
rm -rf $dirs
