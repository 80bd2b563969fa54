#!/bin/bash
# GPU-box A/B (measurement only): batch-1 encoder / postnet per-call time (tools/postnet_bench.py,
# T = 222, L = 100) for the default library and each abvar/lib_*.so, interleaved three times.
set -o pipefail
for k in 1 2 3; do
  for lib in "" abvar/lib_*.so; do
    echo "${lib:-default}: $(env ${lib:+TTS_HIP_LIB=$PWD/$lib} timeout -k 10 120 python tools/postnet_bench.py 222 100 2>&1 | tail -1 | cut -c1-80)" || exit 1
  done
done
