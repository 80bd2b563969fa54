#!/bin/bash
# GPU-box helper: the resident batch decoder (B = 2, 4; mask off, 1000-step cap) under first-poll
# delay settings (tools/resident_batch_bench.py); one JSON line per case, prefixed by the setting.
set -o pipefail
for envs in "TTS_NONE=1" "TTS_RB_SLEEP_HATT=2" "TTS_RB_SLEEP_HDEC=3" "TTS_RB_SLEEP_HDEC=6" "TTS_RB_SLEEP_PRE2=2" \
            "TTS_RB_SLEEP_CTX=2" "TTS_RB_SLEEP_HDEC=3 TTS_RB_SLEEP_PRE2=2"; do
  env $envs timeout -k 10 200 python tools/resident_batch_bench.py --batches 2,4 --cap 1000 --mask off --quick 2>/dev/null \
    | sed "s/^/$envs /" || { echo "$envs failed"; exit 1; }
done
