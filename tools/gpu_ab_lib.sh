#!/bin/bash
# GPU-box A/B (measurement only): the default library vs $VARIANT (a .so built beside it), bench
# line at configs[1] three times each, interleaved.
set -o pipefail
for k in 1 2 3; do
  for lib in "" "$VARIANT"; do
    env ${lib:+TTS_HIP_LIB=$PWD/$lib} timeout -k 10 200 python bench.py --no-cpu-baseline --no-share --no-profile > gpurun_out/ab.json 2> gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
    echo "${lib:-default}: $(python -c "import json;d=json.loads(open('gpurun_out/ab.json').read().strip().splitlines()[-1]);print(round(d['value']), d['stages_rank0'])")"
  done
done
