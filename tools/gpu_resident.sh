#!/bin/bash
# GPU-box helper: resident-decoder tests first (new persistent kernel), then the parity suite.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resident.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_resident.log 2>&1 || { echo resident tests failed; tail -60 gpurun_out/pytest_resident.log; exit 1; }
tail -3 gpurun_out/pytest_resident.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_parity.log 2>&1 || { echo parity failed; tail -60 gpurun_out/pytest_parity.log; exit 1; }
tail -3 gpurun_out/pytest_parity.log
