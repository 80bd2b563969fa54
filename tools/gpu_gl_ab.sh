#!/bin/bash
# GPU-box: Griffin-Lim parity tests (persistent, fused, batched forms), then the batch-1
# persistent loop time and frame-100 phase timers at 222 frames (one workgroup per CU) and 300
# (two per CU) for the default library and each abvar/lib_*.so, interleaved twice.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coresidency.py tests/test_gpu_batched.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "griffin or persistent or synthesize or sensitivity or overlap or gl_ or config4 or wave" > gpurun_out/pt_gl.log 2>&1 || { echo GL tests failed; grep -E "FAILED|Error" gpurun_out/pt_gl.log | head; tail -30 gpurun_out/pt_gl.log; exit 1; }
  tail -1 gpurun_out/pt_gl.log
fi
for k in 1 2; do
  for lib in "" abvar/lib_*.so; do
    for F in 222 300; do
      echo "${lib:-default} F=$F: $(env ${lib:+TTS_HIP_LIB=$PWD/$lib} GL_F=$F TTS_GL_PHASES=100 timeout -k 10 120 python tools/gl_phases_b1.py 2>&1 | grep -E "PHASES|persistent" | tail -2 | tr '\n' ' ' | sed 's/TTS_GL_PHASES frame 100, us per iteration://')" || exit 1
    done
  done
done
