"""Print the kernel timeline of one bench step from a rocprofv3 kernel trace (csv): the K-th
occurrence of an anchor kernel, from the previous step's last GL kernel to this step's."""
import csv
import sys

path = sys.argv[1]
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
anchors = [i for i, r in enumerate(rows) if "encoder_resident_kernel" in r["Kernel_Name"]]
ends = [i for i, r in enumerate(rows) if "preemph_scan_kernel" in r["Kernel_Name"]]
a = anchors[k]
prev = max([e for e in ends if e < a] or [0])
nxt = min([e for e in ends if e > a])
t0 = int(rows[prev]["End_Timestamp"])
pe = t0
busy = 0
for r in rows[prev + 1:nxt + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} gap {(s - pe) / 1e3:6.1f}  {r['Kernel_Name'][:70]}")
    pe = max(pe, e)
print(f"span {(pe - t0) / 1e3:.1f} us, kernels {busy / 1e3:.1f} us")
