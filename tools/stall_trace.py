#!/usr/bin/env python3
"""Post-decoder per-launch stall (measurement only): from a rocprofv3 --kernel-trace run of
tools/b1_trace.py, the median duration of each kernel of the batch-1 sentence by its position
relative to the resident decoder launch (encoder side before it, postnet / Griffin-Lim after).

    python tools/stall_trace.py <rocprof output dir> [label]
"""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
label = sys.argv[2] if len(sys.argv) > 2 else d
kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)[0]
raw = list(csv.DictReader(open(kt)))
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
               "scr %s lds %s vgpr %s/%s sgpr %s grid %s wg %s" % (r.get("Scratch_Size"), r.get("LDS_Block_Size"),
                                                       r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("SGPR_Count"),
                                                       r.get("Grid_Size"), r.get("Workgroup_Size"))) for r in raw)
dec = [i for i, r in enumerate(rows) if "resident_decoder_kernel" in r[2]]
per = {}
for j, i in enumerate(dec[5:-1]):  # skip warm-up sentences
    nxt = dec[5 + j + 1]
    prev = dec[5 + j - 1] if j + 5 > 0 else 0
    # kernels between the previous sentence's preemph and the next decoder
    for off in range(-8, 14):
        k = i + off
        if k <= prev or k >= nxt:
            continue
        s, e, n, res = rows[k]
        short = n.replace("void ", "").replace("tts::", "").replace("(anonymous namespace)::", "").split("(")[0][:34]
        short = short + " | " + res
        gap = (s - rows[k - 1][1]) / 1e3
        per.setdefault((off, short), []).append(((e - s) / 1e3, gap))
print(f"== {label}")
for (off, n), v in sorted(per.items()):
    du = statistics.median(x[0] for x in v)
    ga = statistics.median(x[1] for x in v)
    print(f"{off:+3d} {n:90s} dur {du:8.1f} us  gap {ga:7.1f} us  (n={len(v)})")
