"""ctypes loader of the CPU oracle (oracle/liboracle.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline use this.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from gf_orb_slam_amd.orb import KEYPOINT_DTYPE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_PATH = os.path.join(ROOT, "oracle", "liboracle.so")
_orc = None


def orc() -> ctypes.CDLL:
    global _orc
    if _orc is None:
        _orc = ctypes.CDLL(ORACLE_PATH)
        _orc.orc_fast_atan2.restype = ctypes.c_float
        _orc.orc_fast_atan2.argtypes = [ctypes.c_float, ctypes.c_float]
    return _orc


def _p(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else None


def extract(img: np.ndarray, nfeatures=1000, scale=1.2, nlevels=8, fast_th=20):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    cap = nfeatures + 64
    kps = np.zeros(cap, KEYPOINT_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_int()
    rc = orc().orc_extract(_p(img), w, h, w, nfeatures, ctypes.c_float(scale), nlevels, fast_th, _p(kps),
                           _p(desc), cap, ctypes.byref(n))
    assert rc == 0, rc
    return kps[:n.value].copy(), desc[:n.value].copy()


def level(img: np.ndarray, lvl: int, which: int, nfeatures=1000, scale=1.2, nlevels=8):
    img = np.ascontiguousarray(img, np.uint8)
    h, w = img.shape
    lw, lh = ctypes.c_int(), ctypes.c_int()
    orc().orc_extract_level(_p(img), w, h, nfeatures, ctypes.c_float(scale), nlevels, lvl, which, None,
                            ctypes.byref(lw), ctypes.byref(lh))
    out = np.zeros((lh.value, lw.value), np.uint8)
    orc().orc_extract_level(_p(img), w, h, nfeatures, ctypes.c_float(scale), nlevels, lvl, which, _p(out),
                            ctypes.byref(lw), ctypes.byref(lh))
    return out


def plan(w, h, nfeatures=1000, scale=1.2, nlevels=8):
    lw = np.zeros(nlevels, np.int32)
    lh = np.zeros(nlevels, np.int32)
    fpl = np.zeros(nlevels, np.int32)
    sc = np.zeros(nlevels, np.float32)
    um = np.zeros(16, np.int32)
    orc().orc_extractor_plan(w, h, nfeatures, ctypes.c_float(scale), nlevels, _p(lw), _p(lh), _p(fpl), _p(sc),
                             _p(um))
    return lw, lh, fpl, sc, um
