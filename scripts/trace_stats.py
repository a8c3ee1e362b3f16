"""Per-kernel duration statistics from a rocprofv3 --kernel-trace CSV, for the
dispatches of one launch shape only (Grid_Size_Y = frames per launch, e.g.
the 256-sequence group launches of bench.py's timed region — the same
command's start-up work launches the extraction kernels on single frames).
Usage: python scripts/trace_stats.py <run_kernel_trace.csv> <grid_y> [out.csv]"""
import collections
import csv
import re
import sys

gy = int(sys.argv[2])
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if int(r["Grid_Size_Y"]) != gy:
        continue
    name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
    acc[name].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
rows = sorted(((k, v) for k, v in acc.items()), key=lambda kv: -sum(kv[1]))
out = open(sys.argv[3], "w") if len(sys.argv) > 3 else sys.stdout
w = csv.writer(out)
w.writerow(["Name", "Grid_Size_Y", "Calls", "TotalDurationNs", "AverageNs", "MinNs", "MaxNs"])
for k, v in rows:
    w.writerow([k, gy, len(v), sum(v), round(sum(v) / len(v), 1), min(v), max(v)])
