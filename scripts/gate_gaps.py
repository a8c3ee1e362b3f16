"""Extraction-gate hand-over gaps from a rocprofv3 kernel trace of bench.py.

For every group step (k_fe_begin), the time from the previous group's
k_describe end (the gate's done event) to this k_fe_begin start, and which
kernel ended last before it. Usage: python scripts/gate_gaps.py TRACE.csv
"""
import csv
import json
import sys

import numpy as np


def main(path: str) -> None:
    ev = []
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            if n in ("k_fe_begin", "k_describe", "k_fe_end"):
                ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Queue_Id"]))
    ev.sort()
    begs = [x for x in ev if x[2] == "k_fe_begin"]
    descs = [x for x in ev if x[2] == "k_describe"]
    ends = [d[1] for d in descs]
    gaps, periods = [], []
    last_b = None
    for b in begs:
        i = np.searchsorted(ends, b[0], side="right") - 1
        if i >= 0 and descs[i][3] != b[3]:
            gaps.append((b[0] - descs[i][1]) / 1e3)
        if last_b is not None:
            periods.append((b[0] - last_b) / 1e3)
        last_b = b[0]
    g = np.array(gaps[len(gaps) // 3:])  # after warm-up
    p = np.array(periods[len(periods) // 3:])
    out = {"handovers": int(g.size), "gap_us_median": round(float(np.median(g)), 1),
           "gap_us_p90": round(float(np.percentile(g, 90)), 1), "gap_us_min": round(float(g.min()), 1),
           "begin_period_us_median": round(float(np.median(p)), 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1])
