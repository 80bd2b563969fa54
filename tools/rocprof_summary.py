#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run (kernel_stats.csv) as a fixed-width table."""
import csv
import sys


def main(path, out=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    lines = [f"{'kernel':96s} {'calls':>7s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'total_ms':>9s} {'pct':>6s}"]
    for r in rows:
        lines.append(f"{r['Name'][:96]:96s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:9.2f} "
                     f"{float(r['MinNs'])/1e3:9.2f} {float(r['MaxNs'])/1e3:9.2f} "
                     f"{float(r['TotalDurationNs'])/1e6:9.2f} {float(r['Percentage']):6.2f}")
    txt = "\n".join(lines) + "\n"
    if out:
        open(out, "w").write(txt)
    print(txt)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
