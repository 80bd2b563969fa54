"""Per-kernel mean durations and the sentence period from rocprofv3 kernel traces of tools/b1_trace.py
(measurement only): python tools/b1_kernel_ab.py <trace dir> [<trace dir> ...]"""
import csv
import glob
import statistics
import sys
from collections import defaultdict

res = {}
for d in sys.argv[1:]:
    kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kt)))
    enc = [s for s, e, n in rows if "encoder_resident_kernel" in n]
    per = [(b - a) / 1e3 for a, b in zip(enc[5:], enc[6:])]
    dur = defaultdict(list)
    t_lo = enc[5]
    for s, e, n in rows:
        if s >= t_lo:
            dur[n[:60]].append((e - s) / 1e3)
    res[d] = (statistics.median(per) if per else 0, {k: (statistics.mean(v), len(v)) for k, v in dur.items()})
names = sorted({k for _, (p, m) in res.items() for k in m}, key=lambda k: -max(res[d][1].get(k, (0, 0))[0] * res[d][1].get(k, (0, 1))[1] for d in res))
print("sentence period (median us):", {d: round(p, 1) for d, (p, m) in res.items()})
for k in names[:30]:
    print(f"{k:62s}", " ".join(f"{res[d][1].get(k, (0, 0))[0]:9.1f} x{res[d][1].get(k, (0, 0))[1]:4d}" for d in res))
