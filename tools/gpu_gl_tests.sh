set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_coresidency.py tests/test_gpu_batched.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "griffin or synthesize or persistent or overlap or config or timeout or long" > gpurun_out/pt_gl.log 2>&1 || { echo tests failed; grep -E "FAIL|Error|assert" gpurun_out/pt_gl.log | head -20; tail -40 gpurun_out/pt_gl.log; exit 1; }
tail -2 gpurun_out/pt_gl.log
TTS_GL_PHASES=100 timeout -k 10 200 python bench.py --no-cpu-baseline --no-profile > gpurun_out/bench_gl.json 2> gpurun_out/bench_gl.err; grep PHASES gpurun_out/bench_gl.err | tail -2; python tools/bench_digest.py gpurun_out/bench_gl.json
