"""Per-kernel statistics of the 256-frame dispatches (grid y = 256) in a
rocprofv3 kernel trace: the launches the bench's timed region is made of
(its warm-up included), as a csv like run_kernel_stats.csv.
Usage: python scripts/trace_group.py run_kernel_trace.csv [grid_y] > out.csv"""
import csv
import sys
from collections import defaultdict

gy = sys.argv[2] if len(sys.argv) > 2 else "256"
acc = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if r.get("Grid_Size_Y") != gy:
        continue
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
    acc[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in acc.values())
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([k, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / tot, 2), min(v), max(v)])
