#!/bin/bash
# GPU-box helper for iteration: a pytest selection (PYTEST_K), then bench lines for each BENCH_CASES
# entry (';'-separated bench.py argument lists).  Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
if [ -n "${PYTEST_K}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "${PYTEST_K}" > gpurun_out/pytest_quick.log 2>&1 || { echo tests failed; tail -60 gpurun_out/pytest_quick.log; exit 1; }
  tail -3 gpurun_out/pytest_quick.log
fi
i=0
IFS=';' read -ra CASES <<< "${BENCH_CASES}"
for c in "${CASES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline $c > gpurun_out/quick_$i.json 2> gpurun_out/quick_$i.err \
    || { echo "bench $c failed"; tail -30 gpurun_out/quick_$i.err; exit 1; }
  echo "== $c"; python tools/bench_digest.py gpurun_out/quick_$i.json
done
