"""Scan gfx950 assembly (hipcc --cuda-device-only -S) for vector
instructions placed in a join block before that block's exec restore
(`s_or_b64 exec, exec, s[..]`). Such an instruction runs under the mask of
the branch that just ended, so lanes outside it keep stale register values:
the miscompile that broke k_active_match's RNG state under register pressure
(spill copies to AGPRs of a loop-carried value). Prints every
occurrence per kernel; exit status 1 when any kernel named on the command
line (default: all) has one.
Usage: python scripts/isa_exec_check.py FILE.s [kernel-substring ...]"""
import re
import sys


def scan(path):
    kern, out = None, {}
    block = []
    for ln in open(path):
        s = ln.strip()
        m = re.match(r"^(_Z\S+):", s)
        if m:
            kern, block = m.group(1), []
            continue
        if kern is None:
            continue
        if re.match(r"^\.LBB\S+:", s) or s.startswith("; %bb."):
            block = []
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        if re.match(r"s_or_b64 exec, exec, s\[\d+:\d+\]", s):
            bad = [b for b in block if b.startswith("v_")]
            if bad:
                out.setdefault(kern, []).append(bad)
            block = []
            continue
        if s.startswith("s_cbranch") or s.startswith("s_branch") or "saveexec" in s or s.startswith("s_endpgm"):
            block = []
            continue
        block.append(s)
    return out


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    res = scan(path)
    bad = 0
    for k, occ in res.items():
        if pats and not any(p in k for p in pats):
            continue
        bad += 1
        print(f"{k}: {len(occ)} join block(s) with vector instructions before the exec restore")
        for o in occ[:6]:
            print("   ", " | ".join(o[:6]))
    print("clean" if not bad else f"{bad} kernel(s) affected")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
