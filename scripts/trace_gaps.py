"""Graph-replay breakdown from a rocprofv3 kernel trace: the last N steps'
kernels (the step is bracketed by k_fe_begin), busy time vs span.
Usage: python scripts/trace_gaps.py run_kernel_trace.csv [N]"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
for r in rows:
    r["Kernel_Name"] = r["Kernel_Name"].replace("(anonymous namespace)::", "")
N = int(sys.argv[2]) if len(sys.argv) > 2 else 50
starts = [i for i, r in enumerate(rows) if r["Kernel_Name"].split("(")[0].endswith("k_fe_begin")]
sel = rows[starts[-N - 1]:starts[-1]]
span = (int(rows[starts[-1]]["Start_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / N / 1e3
busy = defaultdict(float)
cnt = defaultdict(int)
for r in sel:
    k = r["Kernel_Name"].split("(")[0].split("::")[-1].split("<")[0]
    busy[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / N / 1e3
    cnt[k] += 1
gaps = [(int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3 for a, b in zip(sel, sel[1:])]
print(f"span per step {span:.1f} us, kernel busy {sum(busy.values()):.1f} us, launches per step {len(sel) / N:.1f}, "
      f"mean gap {sum(gaps) / len(gaps):.2f} us")
for k, v in sorted(busy.items(), key=lambda kv: -kv[1]):
    print(f"  {k:28s} {v:8.1f} us  x{cnt[k] / N:.0f}")
