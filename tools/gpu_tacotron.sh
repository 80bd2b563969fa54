#!/bin/bash
# GPU-box helper: Tacotron / TacotronGST parity tests (one process, per-test timeout).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_tacotron.py -x -v --timeout 180 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_tacotron.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_tacotron.log
exit $rc
