"""Per-kernel averages of rocprofv3 --pmc passes (scripts/pmc_extract.sh):
python scripts/pmc_summary.py gpurun_out/<tag> [kernel ...]"""
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
        per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (name, _, ctr), v in per.items():
        acc[name][ctr].append(v)
out = {}
for name, ctrs in acc.items():
    if want and name not in want:
        continue
    out[name] = {c: sum(v) / len(v) for c, v in ctrs.items()}
    out[name]["dispatches"] = max(len(v) for v in ctrs.values())
print(json.dumps(out, indent=1, sort_keys=True))
