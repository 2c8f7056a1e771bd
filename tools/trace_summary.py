"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel count / mean / median
duration and the mean idle gap before each kernel (development aid)."""
import csv
import statistics
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = defaultdict(list)
gap = defaultdict(list)
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    dur[name].append((e - s) / 1000)
    if prev_end is not None and s >= prev_end:
        gap[name].append((s - prev_end) / 1000)
    prev_end = e
tot = sum(sum(v) for v in dur.values())
print(f"{'kernel':40s} {'calls':>7s} {'mean_us':>9s} {'med_us':>9s} {'gap_us':>8s} {'share':>6s}")
for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    g = statistics.mean(gap[k]) if gap[k] else 0
    print(f"{k[:40]:40s} {len(v):7d} {statistics.mean(v):9.2f} {statistics.median(v):9.2f} {g:8.2f} {100*sum(v)/tot:5.1f}%")
