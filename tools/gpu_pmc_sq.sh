#!/bin/bash
# GPU-box helper: kernel trace + one SQ counter pass over a short bench run (BENCH_ARGS), summarised
# per kernel into gpurun_out/sq_summary.txt.  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/kt -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} > $R/gpurun_out/kt.json 2> $R/gpurun_out/kt.err
echo "kernel trace rc=$?"
timeout -s KILL 300 rocprofv3 --pmc ${SQ_COUNTERS:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES} \
  -d $R/gpurun_out/sq -o run --output-format csv -- \
  python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} > $R/gpurun_out/sq.json 2> $R/gpurun_out/sq.err
echo "pmc rc=$?"
cd $R && python3 tools/sq_summary.py gpurun_out/kt gpurun_out/sq > gpurun_out/sq_summary.txt; head -40 gpurun_out/sq_summary.txt
