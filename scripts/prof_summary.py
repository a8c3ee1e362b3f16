"""rocprofv3 --stats kernel summary (run_kernel_stats.csv) -> markdown table.
Usage: python scripts/prof_summary.py <run_kernel_stats.csv> [top]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
print("| kernel | calls | avg us | min us | max us | total ms | % |")
print("|---|---|---|---|---|---|---|")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
    name = re.sub(r"\(anonymous namespace\)::", "", r["Name"]).split("(")[0]
    print(f"| {name} | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
          f"{float(r['MaxNs']) / 1e3:.1f} | {float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.2f} |")
