#!/bin/bash
# GPU-box helper: alternate configs[1] per-sentence timings (tools/b1_ab.py) over "name|ENV=... lib"
# cases given one per line in $CASES (lib relative to the repo root).  Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2 3; do
  while IFS='|' read -r name envs lib; do
    [ -z "$name" ] && continue
    r=$(env $envs TTS_HIP_LIB=$PWD/$lib timeout -k 10 120 python tools/b1_ab.py 2>/dev/null) || { echo "$name failed"; exit 1; }
    echo "$rep $name $r"
  done <<< "$CASES"
done
