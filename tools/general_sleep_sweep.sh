#!/bin/bash
# GPU-box helper: the batch-1 general resident form (Synthesizer configuration and the location +
# softmax default) under first-poll delay settings; one line per setting (tools/resident_general_b1.py).
set -o pipefail
for envs in "TTS_NONE=1" "TTS_RES_SLEEP_HATT=0 TTS_RES_SLEEP_HDEC=0 TTS_RES_SLEEP_PRE2=0" \
            "TTS_RES_SLEEP_HATT=3 TTS_RES_SLEEP_HDEC=3" "TTS_RES_SLEEP_HATT=7 TTS_RES_SLEEP_HDEC=7" \
            "TTS_RES_SLEEP_CTX=2" "TTS_RES_SLEEP_P1=2"; do
  r=$(env $envs TTS_CONFIGS=server_fwd_sigmoid_nomask,default_loc_softmax,synthesize_fwd_sigmoid_mask \
      timeout -k 10 200 python tools/resident_general_b1.py 2>/dev/null) || { echo "$envs failed"; exit 1; }
  echo "$envs $r"
done
