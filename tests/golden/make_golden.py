"""Regenerates the extraction golden fixtures from the CPU oracle.

Frames are small seeded synthetic images (stored as .npy so the fixture does
not depend on the generator staying bit-stable); digests pin the oracle's
keypoints (28-byte cv::KeyPoint records) and descriptors.
Run: python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, os.path.dirname(HERE))

import oracle_lib as O  # noqa: E402
from gf_orb_slam_amd import synth  # noqa: E402

cases = []
for name, (w, h, nf, seed) in {"frame_320x240_s1.npy": (320, 240, 500, 1),
                               "frame_400x300_s2.npy": (400, 300, 800, 2)}.items():
    img = synth.synth_frame(w, h, seed, n_shapes=120)
    np.save(os.path.join(HERE, name), img)
    k, d = O.extract(img, nfeatures=nf)
    cases.append({"frame": name, "nfeatures": nf, "n": int(len(k)),
                  "kps_sha256": hashlib.sha256(k.tobytes()).hexdigest(),
                  "desc_sha256": hashlib.sha256(d.tobytes()).hexdigest()})
json.dump({"generator": "tests/golden/make_golden.py", "cases": cases},
          open(os.path.join(HERE, "extract_golden.json"), "w"), indent=1)
print(cases)
