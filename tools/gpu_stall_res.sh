set -o pipefail
R=$(pwd); mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
TTS_COOP=0 timeout -k 10 120 rocprofv3 --kernel-trace -d $R/gpurun_out/st_b -o run --output-format csv -- python3 $R/tools/b1_trace.py > $R/gpurun_out/st_b.log 2>&1 || exit 1
python3 $R/tools/stall_trace.py $R/gpurun_out/st_b base > $R/gpurun_out/stall_res.txt; rm -rf $R/gpurun_out/st_b; cat $R/gpurun_out/stall_res.txt
