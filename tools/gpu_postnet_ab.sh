#!/bin/bash
# GPU-box helper: tools/postnet_bench.py under each "ENV=..." line of $CASES.  Run from the repo root.
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
while IFS= read -r envs; do
  [ -z "$envs" ] && continue
  env $envs timeout -k 10 120 python tools/postnet_bench.py 2>&1 | grep "us per call" || { echo "$envs failed"; exit 1; }
done <<< "$CASES"
done
