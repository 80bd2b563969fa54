#!/bin/bash
# GPU-box helper: configs[1] measurement set on the current tree -> gpurun_out/: rocprofv3 kernel
# statistics of a short bench run (r_b1_kernel_stats.txt) and the FETCH_SIZE / WRITE_SIZE passes
# (separate runs) summarised per launch by tools/pmc_summary.py (pmc_b1.json).  Run from the repo root.
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-share"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/ks -o run --output-format csv -- python3 $B > $R/gpurun_out/ks.log 2>&1 || { echo "stats failed"; tail -5 $R/gpurun_out/ks.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $R/gpurun_out/pf -o run --output-format csv -- python3 $B > $R/gpurun_out/pf.log 2>&1 || { echo "fetch pass failed"; tail -5 $R/gpurun_out/pf.log; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $R/gpurun_out/pw -o run --output-format csv -- python3 $B > $R/gpurun_out/pw.log 2>&1 || { echo "write pass failed"; tail -5 $R/gpurun_out/pw.log; exit 1; }
cd $R
python3 tools/rocprof_summary.py $(find gpurun_out/ks -name "*kernel_stats.csv" | head -1) gpurun_out/r_b1_kernel_stats.txt > /dev/null
python3 tools/pmc_summary.py $(find gpurun_out/pf -name "*counter_collection.csv" | head -1) $(find gpurun_out/pw -name "*counter_collection.csv" | head -1) gpurun_out/pmc_b1.json > /dev/null
rm -rf gpurun_out/ks gpurun_out/pf gpurun_out/pw
cut -c1-100,190- gpurun_out/r_b1_kernel_stats.txt | sed -n 1,8p
python3 -c "import json; d=json.load(open('gpurun_out/pmc_b1.json'))['per_launch_hbm_bytes']; print({k: round(v/1e6,2) for k,v in d.items() if k.startswith(('resident','gl_pers'))})"
