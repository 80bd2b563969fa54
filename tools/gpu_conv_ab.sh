#!/bin/bash
# GPU-box A/B (measurement only): batch-1 postnet / encoder time per call (tools/postnet_bench.py)
# for the default library and every variants/lib_*.so, interleaved twice.
set -o pipefail
for k in 1 2; do
  for lib in "" variants/lib_*.so; do
    echo "${lib:-default}: $(env ${lib:+TTS_HIP_LIB=$PWD/$lib} timeout -k 10 100 python tools/postnet_bench.py 222 100 2>&1 | tail -1)" || exit 1
  done
done
