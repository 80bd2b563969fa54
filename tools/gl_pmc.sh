set -o pipefail
R=$(pwd); mkdir -p gpurun_out; cd /tmp && export TMPDIR=/tmp
for P in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU" "TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace -d $R/gpurun_out/pmc$n -o run --output-format csv -- python3 $R/tools/gl_run_once.py 64 > $R/gpurun_out/pmc$n.log 2>&1 || { echo "pmc pass $n failed"; tail -5 $R/gpurun_out/pmc$n.log; exit 1; }
done
cd $R && python3 - <<'PY'
import csv,glob
from collections import defaultdict
for n in (1,2):
    f=sorted(glob.glob(f'gpurun_out/pmc{n}/**/*counter_collection.csv',recursive=True))[0]
    acc=defaultdict(lambda: defaultdict(float)); cnt=defaultdict(set)
    for r in csv.DictReader(open(f)):
        k=r['Kernel_Name']
        if 'gl_iter_wave' not in k and 'gl_ola' not in k: continue
        acc[k][r['Counter_Name']]+=float(r['Counter_Value']); cnt[k].add(r['Dispatch_Id'])
    for k,d in acc.items():
        print(k[:40], {c: round(v/len(cnt[k])) for c,v in d.items()})
PY
rm -rf gpurun_out/pmc1 gpurun_out/pmc2
