"""Per-kernel duration outliers in a rocprofv3 kernel trace (csv): for every kernel name, the median
duration and how many launches took more than median + 20 us (the sporadic ~35-40 us stalls)."""
import csv
import glob
import statistics
import sys

kt = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
by = {}
for r in csv.DictReader(open(kt)):
    by.setdefault(r["Kernel_Name"][:70], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
tot_extra = 0.0
for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
    med = statistics.median(v)
    out = [x for x in v if x > med + 20]
    tot_extra += sum(x - med for x in out)
    if out:
        print(f"{len(v):5d} med {med:8.1f} outliers {len(out):4d} mean_excess {statistics.mean(out) - med:7.1f}  {k}")
print(f"total outlier excess {tot_extra:.0f} us")
# which kernel ran right before each outlier (time order), counted
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:50]) for r in csv.DictReader(open(kt))))
meds = {k[:50]: statistics.median(v) for k, v in by.items()}
prev = {}
for i in range(1, len(rows)):
    s, e, n = rows[i]
    if (e - s) / 1e3 > meds[n] + 20:
        key = (rows[i - 1][2], n, round((s - rows[i - 1][1]) / 1e3))
        prev[key[:2]] = prev.get(key[:2], 0) + 1
for (p, n), c in sorted(prev.items(), key=lambda kv: -kv[1])[:12]:
    print(f"{c:4d}  after {p:50s} -> {n}")
# idle gap (us) before outliers vs before normal launches of the same kernels
g_out, g_norm = [], []
for i in range(1, len(rows)):
    s, e, n = rows[i]
    gap = (s - max(r[1] for r in rows[max(0, i - 4):i])) / 1e3
    (g_out if (e - s) / 1e3 > meds[n] + 20 else g_norm).append(gap)
q = lambda v, p: sorted(v)[int(p * (len(v) - 1))] if v else float("nan")
print("gap before outliers: n %d median %.1f p90 %.1f | before normal: n %d median %.1f p90 %.1f" % (
    len(g_out), q(g_out, .5), q(g_out, .9), len(g_norm), q(g_norm, .5), q(g_norm, .9)))
big = [i for i in range(1, len(rows)) if (rows[i][0] - rows[i - 1][1]) / 1e3 > 15]
nb = sum(1 for i in big if (rows[i][1] - rows[i][0]) / 1e3 > meds[rows[i][2]] + 20)
print("launches after an idle gap > 15 us: %d, of them outliers: %d" % (len(big), nb))
