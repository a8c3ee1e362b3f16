"""Extraction chain of every group step in a rocprofv3 kernel trace of
bench.py: per position (k_fe_begin .. k_describe on the group's queue) the
kernel's mean duration and the mean gap before it, and the hand-over gap from
the previous group's k_describe end. Usage: python scripts/chain_gaps.py TRACE.csv"""
import collections
import csv
import sys

CHAIN_END = "k_describe"


def main(path):
    rows = []
    rd = csv.DictReader(open(path))
    qcol = "Queue_Id" if "Queue_Id" in rd.fieldnames else ("Stream_Id" if "Stream_Id" in rd.fieldnames else None)
    print("columns:", rd.fieldnames)
    for r in rd:
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
        n = n.split("<")[0].replace("void ", "").strip()
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r[qcol] if qcol else "0"))
    print("kernel names:", collections.Counter(x[2] for x in rows).most_common(12))
    rows.sort()
    byq = collections.defaultdict(list)
    for x in rows:
        byq[x[3]].append(x)
    chains = []
    for q, ev in byq.items():
        i = 0
        while i < len(ev):
            if ev[i][2] == "k_fe_begin":
                j = i
                seq = []
                while j < len(ev) and ev[j][2] != CHAIN_END:
                    seq.append(ev[j])
                    j += 1
                if j < len(ev):
                    seq.append(ev[j])
                    chains.append(seq)
                i = j + 1
            else:
                i += 1
    # keep the chains of the batch shape that dominates (the timed groups)
    lens = collections.Counter(len(c) for c in chains)
    L = lens.most_common(1)[0][0]
    chains = [c for c in chains if len(c) == L]
    chains.sort(key=lambda c: c[0][0])
    dur = collections.defaultdict(list)
    gap = collections.defaultdict(list)
    for c in chains:
        for k, e in enumerate(c):
            dur[(k, e[2])].append((e[1] - e[0]) / 1e3)
            if k:
                gap[(k, e[2])].append((e[0] - c[k - 1][1]) / 1e3)
    print(f"{len(chains)} chains of {L} kernels (k_fe_begin .. {CHAIN_END})")
    tot_d = tot_g = 0.0
    for key in sorted(dur):
        d = sum(dur[key]) / len(dur[key])
        g = sum(gap[key]) / len(gap[key]) if gap[key] else 0.0
        tot_d += d
        tot_g += g
        print(f"  {key[0]:2d} {key[1]:24s} dur {d:8.1f} us  gap before {g:7.1f} us")
    span = sum((c[-1][1] - c[0][0]) / 1e3 for c in chains) / len(chains)
    print(f"chain span {span:.1f} us = kernels {tot_d:.1f} + gaps {tot_g:.1f}")
    # hand-over: previous chain's end (any queue) to this chain's start
    ho = [(chains[i][0][0] - chains[i - 1][-1][1]) / 1e3 for i in range(1, len(chains))]
    ho.sort()
    if ho:
        print(f"hand-over gap median {ho[len(ho) // 2]:.1f} us, mean {sum(ho) / len(ho):.1f} us, p90 {ho[int(0.9 * len(ho))]:.1f} us")


if __name__ == "__main__":
    main(sys.argv[1])
