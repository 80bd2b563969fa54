#!/bin/bash
# GPU-box helper: configs[4] (bench.py --model gst) under TacotronGST resident-decoder first-poll delays
set -o pipefail
for v in 0 2 4 8; do
  r=$(TTS_TACO_FIRST_SLEEP=$v timeout -k 10 300 python bench.py --model gst --steps 3 --warmup 1 2>/dev/null | tail -1) || { echo "$v failed"; exit 1; }
  echo "$v $r"
done
