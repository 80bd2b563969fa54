"""Print one configs[1] step's kernels and memory copies (rocprofv3 --kernel-trace --memory-copy-trace
csv files) in time order, relative to the step's encoder-resident launch (anchor K)."""
import csv
import glob
import sys

d = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
mt = glob.glob(d + "/**/*memory_copy_trace.csv", recursive=True)
rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K " + r["Kernel_Name"][:60]) for r in csv.DictReader(open(kt))]
if mt:
    for r in csv.DictReader(open(mt[0])):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
                     "C %s %s bytes" % (r.get("Direction", r.get("Operation", "?")), r.get("Bytes", r.get("Size", "?")))))
rows.sort()
anch = [i for i, r in enumerate(rows) if "encoder_resident_kernel" in r[2]]
a, b = anch[k], anch[k + 1]
t0 = rows[a][0]
lo = max(i for i in range(a) if "preemph" in rows[i][2])
hi = max(i for i in range(b) if "preemph" in rows[i][2])
pe = rows[lo][1]
for s, e, n in rows[lo:hi + 1]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:7.1f} gap {(s - pe) / 1e3:6.1f}  {n}")
    pe = max(pe, e)
