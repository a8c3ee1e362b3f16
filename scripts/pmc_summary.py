"""Per-kernel averages of rocprofv3 --pmc passes (scripts/pmc_extract.sh):
python scripts/pmc_summary.py <dir> [kernel ...]

Dispatches of one kernel with different grid sizes (e.g. the batch-1
extraction calls that build the maps next to the 256-frame ones) are kept
apart: each kernel reports the dispatches of its largest grid only."""
import collections
import csv
import glob
import json
import os
import re
import sys

root = sys.argv[1]
want = sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        name = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0]
        grid = int(r.get("Grid_Size", 0) or 0)
        per[(name, grid, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (name, grid, _, ctr), v in per.items():
        acc[(name, grid)][ctr].append(v)
out = {}
for (name, grid), ctrs in acc.items():
    if want and name not in want:
        continue
    if name in out and out[name]["grid_size"] > grid:
        continue
    out[name] = {c: sum(v) / len(v) for c, v in ctrs.items()}
    out[name]["dispatches"] = max(len(v) for v in ctrs.values())
    out[name]["grid_size"] = grid
print(json.dumps(out, indent=1, sort_keys=True))
