#!/bin/bash
# GPU-box helper: the batch-1 resident decoder (Synthesizer configuration, location + softmax default,
# synthesize.py's masked form) under first-poll delay settings; one line per setting
# (tools/resident_general_b1.py).
set -o pipefail
for envs in "TTS_NONE=1" "TTS_RES_SLEEP_HATT=6" "TTS_RES_SLEEP_HATT=4"; do
  r=$(env $envs TTS_CONFIGS=server_fwd_sigmoid_nomask,default_loc_softmax,synthesize_fwd_sigmoid_mask \
      timeout -k 10 200 python tools/resident_general_b1.py 2>/dev/null | tail -1) || { echo "$envs failed"; exit 1; }
  echo "$envs $r"
done
