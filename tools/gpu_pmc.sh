#!/bin/bash
# GPU-box helper: two separate rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) over a short bench
# run, then per-kernel HBM bytes per launch -> gpurun_out/pmc.json.  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d $R/gpurun_out/pmc_$C -o run --output-format csv -- \
    python $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} \
    > $R/gpurun_out/pmc_$C.json 2> $R/gpurun_out/pmc_$C.err || { echo "pmc $C failed"; tail -20 $R/gpurun_out/pmc_$C.err; exit 1; }
done
python $R/tools/pmc_summary.py $(ls $R/gpurun_out/pmc_FETCH_SIZE/*counter_collection.csv | head -1) \
  $(ls $R/gpurun_out/pmc_WRITE_SIZE/*counter_collection.csv | head -1) $R/gpurun_out/pmc.json
