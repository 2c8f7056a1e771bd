"""Per-kernel-name duration stats of a kernel-trace CSV, split by grid size."""
import csv, statistics, sys
from collections import defaultdict
d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    key = (name, r.get("Grid_Size_X", r.get("Grid_Size", "?")), r.get("Workgroup_Size_X", r.get("Workgroup_Size", "?")))
    d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: (kv[0][0], int(kv[0][2]) if kv[0][2].isdigit() else 0, int(kv[0][1]) if kv[0][1].isdigit() else 0)):
    print(f"{k[0]:30s} grid {k[1]:>8s} wg {k[2]:>5s} n {len(v):5d} mean {statistics.mean(v):8.2f} med {statistics.median(v):8.2f} us")
