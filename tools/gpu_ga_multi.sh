#!/bin/bash
# GPU-box (measurement only): tools/general_attention_b1.py for the default library and every
# variants/lib_*.so.
for lib in "" variants/lib_*.so; do
  echo "${lib:-default}: $(env ${lib:+TTS_HIP_LIB=$PWD/$lib} timeout -k 10 100 python tools/general_attention_b1.py 2>&1 | grep loc_softmax)"
done
