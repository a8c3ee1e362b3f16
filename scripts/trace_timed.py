"""Per-kernel statistics of a bench run's timed region from a rocprofv3
kernel trace: the dispatches between the first k_fe_begin of the timed
steps and the last k_fe_end of them (warm-up W steps and K timed steps of G
stream groups; one k_fe_begin / k_fe_end per group and step), as a csv like
run_kernel_stats.csv.
Usage: python scripts/trace_timed.py run_kernel_trace.csv W K G > out.csv"""
import csv
import sys
from collections import defaultdict

W, K, G = (int(x) for x in sys.argv[2:5])
rows = list(csv.DictReader(open(sys.argv[1])))


def name(r):
    return r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]


beg = sorted(int(r["Start_Timestamp"]) for r in rows if name(r) == "k_fe_begin")
end = sorted(int(r["End_Timestamp"]) for r in rows if name(r) == "k_fe_end")
t0, t1 = beg[W * G], end[(W + K) * G - 1]
acc = defaultdict(list)
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 and e <= t1:
        acc[name(r)].append(e - s)
tot = sum(sum(v) for v in acc.values())
w = csv.writer(sys.stdout)
w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
for k, v in sorted(acc.items(), key=lambda kv: -sum(kv[1])):
    w.writerow([k, len(v), sum(v), round(sum(v) / len(v), 1), round(100.0 * sum(v) / tot, 2), min(v), max(v)])
print(f"# timed region {(t1 - t0) / 1e6:.3f} ms for {K} steps", file=sys.stderr)
