#!/usr/bin/env python3
"""Host/device timeline of one pipelined configs[1] sentence (measurement only): HIP API calls and
kernels from a rocprofv3 --hip-trace --kernel-trace run of tools/b1_trace.py, merged in time order
around the K-th resident decoder launch.

    python tools/host_trace.py <rocprof output dir> [K]
"""
import csv
import glob
import sys

d = sys.argv[1]
K = int(sys.argv[2]) if len(sys.argv) > 2 else 12
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
ht = glob.glob(d + "/**/*hip_api_trace.csv", recursive=True)
ev = []
for r in csv.DictReader(open(kt)):
    n = r["Kernel_Name"].replace("void ", "").replace("tts::", "").replace("(anonymous namespace)::", "").split("(")[0]
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "GPU " + n[:40]))
for r in csv.DictReader(open(ht[0])):
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "    host " + r["Function"]))
ev.sort()
dec = [i for i, e in enumerate(ev) if "resident_decoder_kernel" in e[2]]
a, b = dec[K], dec[K + 1]
t0 = ev[a][1]  # decoder end
for s, e, n in ev[a:b + 1]:
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  {n}")
