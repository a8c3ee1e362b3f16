"""ORBvoc text -> binary converter, the counterpart of the reference's
tools/bin_vocabulary.cc (loadFromTextFile, then saveToBinaryFile). Host only.

    python -m gf_orb_slam_amd.bin_vocabulary ORBvoc.txt ORBvoc.bin
"""
from __future__ import annotations

import sys
import time

from .bow import read_vocabulary, save_vocabulary_binary


def convert(src: str, dst: str) -> dict:
    t0 = time.perf_counter()
    tree = read_vocabulary(src)  # a .txt path takes the text loader
    t1 = time.perf_counter()
    save_vocabulary_binary(tree, dst)
    t2 = time.perf_counter()
    return {"nodes": len(tree["parent"]), "load_s": t1 - t0, "save_s": t2 - t1}


def main(argv: list[str]) -> int:
    if len(argv) != 3:
        print(__doc__)
        return 2
    r = convert(argv[1], argv[2])
    print(f"Loading from text: {r['load_s']:.2f}s\nSaving as binary: {r['save_s']:.2f}s ({r['nodes']} nodes)")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
