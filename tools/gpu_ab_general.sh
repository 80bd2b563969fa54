#!/bin/bash
# GPU-box A/B (measurement only): resident decoder µs/step per attention configuration
# (tools/resident_general_b1.py, resident leg only) for the default library and each abvar/lib_*.so,
# interleaved three times.  CFGS selects the configurations (comma list; default: server + mask).
set -o pipefail
CFGS=${CFGS:-server_fwd_sigmoid_nomask,synthesize_fwd_sigmoid_mask,default_loc_softmax}
for k in 1 2 3; do
  for lib in "" abvar/lib_*.so; do
    r=$(env ${lib:+TTS_HIP_LIB=$PWD/$lib} TTS_CONFIGS=$CFGS TTS_NO_ML=1 timeout -k 10 200 python tools/resident_general_b1.py 2>/dev/null | tail -1) || { echo "run failed: $lib"; exit 1; }
    echo "${lib:-default}: $(python -c "import json,sys;d=json.loads(sys.argv[1]);print({k: v['resident']['us_per_step'] for k, v in d['configs'].items()})" "$r")"
  done
done
