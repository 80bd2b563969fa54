"""Per-kernel mean duration (kernel trace) and mean SQ counter values (one --pmc pass)."""
import csv
import glob
import os
import sys
from collections import defaultdict


def first(pattern):
    g = sorted(glob.glob(pattern, recursive=True))
    return g[0] if g else None


kt = first(os.path.join(sys.argv[1], "**", "*kernel_stats.csv"))
if kt:
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>9s} {'total_ms':>9s}")
    rows = list(csv.DictReader(open(kt)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:14]:
        print(f"{r['Name'][:70]:70s} {r['Calls']:>6s} {float(r['AverageNs']) / 1e3:9.2f} {float(r['TotalDurationNs']) / 1e6:9.2f}")
cc = first(os.path.join(sys.argv[2], "**", "*counter_collection.csv"))
if cc:
    acc = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(cc)):
        acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    names = sorted({c for k in acc.values() for c in k})
    print()
    print(f"{'kernel':60s} " + " ".join(f"{n[3:17]:>14s}" for n in names))
    top = sorted(acc, key=lambda k: -sum(acc[k].get("SQ_WAVE_CYCLES", [0])))[:14]
    for k in top:
        vals = []
        for n in names:
            v = acc[k].get(n, [])
            # per dispatch: counters repeat per dimension/agent row -> sum rows of one dispatch is
            # approximated by total / calls (calls = number of SQ_WAVE_CYCLES rows / 1)
            vals.append(sum(v) / max(1, len(acc[k].get("SQ_WAVE_CYCLES", v)) or 1))
        print(f"{k[:60]:60s} " + " ".join(f"{x:14.4g}" for x in vals))
