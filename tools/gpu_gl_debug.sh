# Griffin-Lim parity on the GPU, persistent loop (default) -- three passes of the GL tests
set -o pipefail
mkdir -p gpurun_out
for i in 1 2 3; do
  timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q -k "griffin_lim" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gl_d$i.log 2>&1 || { tail -5 gpurun_out/gl_d$i.log; grep -h "^E  " gpurun_out/gl_d$i.log | head -4; exit 1; }
  tail -1 gpurun_out/gl_d$i.log
done
