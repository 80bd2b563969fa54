#!/bin/bash
# GPU-box helper: the committed measurement set for one workload.  Run from the repo root:
#   NAME=r02_b64 BENCH_ARGS="--batch 64" [PREFIX=gst_] bash tools/gpu_profile.sh
# 1. bench.py line (default steps/warmup unless BENCH_STEPS is set)   -> gpurun_out/$NAME/bench.json
# 2. rocprofv3 --kernel-trace --stats over a short bench run          -> .../kernel_stats.{csv,txt}
# 3. two separate --pmc passes, FETCH_SIZE then WRITE_SIZE            -> .../pmc.json (HBM bytes/launch)
# Every GPU step has its own time limit; the script stops at the first failure.
# The profiled runs launch the persistent kernels with a plain launch after the occupancy check
# (TTS_COOP=0, the same kernels): rocprofv3 segfaults at process exit after cooperative launches.
set -o pipefail
R=$(pwd)
O=$R/gpurun_out/${NAME:?NAME required}
mkdir -p $O
timeout -k 10 600 python bench.py ${BENCH_STEPS:-} ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err \
  || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-400
cd /tmp && export TMPDIR=/tmp
TTS_COOP=0 timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
  python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} > $O/kt_bench.json 2> $O/kt.err \
  || { echo "kernel trace failed"; tail -20 $O/kt.err; exit 1; }
KS=$(ls $O/kt/*kernel_stats.csv $O/kt/*/*kernel_stats.csv 2>/dev/null | head -1)
cp $KS $O/kernel_stats.csv
python3 $R/tools/rocprof_summary.py $O/kernel_stats.csv $O/kernel_stats.txt > /dev/null
head -14 $O/kernel_stats.txt
for C in FETCH_SIZE WRITE_SIZE; do
  TTS_COOP=0 timeout -k 10 600 rocprofv3 --pmc $C --kernel-trace -d $O/pmc_$C -o run --output-format csv -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-profile ${BENCH_ARGS} \
    > $O/pmc_$C.json 2> $O/pmc_$C.err || { echo "pmc $C failed"; tail -20 $O/pmc_$C.err; exit 1; }
done
F=$(ls $O/pmc_FETCH_SIZE/*counter_collection.csv $O/pmc_FETCH_SIZE/*/*counter_collection.csv 2>/dev/null | head -1)
W=$(ls $O/pmc_WRITE_SIZE/*counter_collection.csv $O/pmc_WRITE_SIZE/*/*counter_collection.csv 2>/dev/null | head -1)
python3 $R/tools/pmc_summary.py $F $W $O/pmc.json ${PREFIX:-}
# the raw counter CSVs are large: keep only the summaries
rm -rf $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE $O/kt
