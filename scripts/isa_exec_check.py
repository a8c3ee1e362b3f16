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


# lane accesses that ignore EXEC (SGPR spill lanes, broadcasts)
LANE_OPS = ("v_readlane", "v_writelane", "v_readfirstlane")


def scan(path):
    """{kernel: [instructions of each flagged block]}. Only blocks that start
    at the target of an `s_cbranch_execz` are checked (the join of a masked
    region's skip and its fall-through); a branch body (a fall-through
    `; %bb.N:` or an `s_cbranch_execnz` target) that ends with the exec
    restore runs under its mask by design."""
    lines = open(path).read().splitlines()
    # join labels: where a branch that skipped a masked region (s_cbranch_execz) lands
    skip_targets = set(re.findall(r"s_cbranch_execz (\.LBB\S+)", "\n".join(lines)))
    kern, out = None, {}
    block, joined, wwm = [], False, False
    for ln in lines:
        s = ln.strip()
        m = re.match(r"^(_Z\S+):", s)
        if m:
            kern, block, joined = m.group(1), [], False
            continue
        if kern is None:
            continue
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            block, joined = [], m.group(1) in skip_targets
            continue
        if s.startswith("; %bb."):
            block, joined = [], False
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        if wwm:  # whole-wave section (exec = all lanes): its copies see every lane
            if re.match(r"s_mov_b64 exec, s\[\d+:\d+\]", s):
                wwm = False
            continue
        if re.match(r"s_or_saveexec_b64 s\[\d+:\d+\], -1", s):
            wwm = True
            continue
        if re.match(r"s_or_b64 exec, exec, s\[\d+:\d+\]", s):
            bad = [b for b in block if b.startswith("v_") and not b.startswith(LANE_OPS)]
            if bad and joined:
                out.setdefault(kern, []).append(bad)
            # what follows the join's first restore runs under the enclosing region
            block, joined = [], False
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
