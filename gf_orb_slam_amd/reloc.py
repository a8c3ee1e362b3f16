"""Host-side mirror of the track-loss matchers of ORB_SLAM::ORBmatcher and of
KeyFrameDatabase::DetectRelocalisationCandidates over libgfslam's C-ABI
(abi.h gf_window_search ... gf_reloc_candidates; csrc/reloc.hip). The
batched tracking step runs the same device code inside its TrackPreviousFrame
and Relocalisation paths; these entry points run one problem each."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr
from .matcher import MAP_POINT_DTYPE
from .orb import KEYPOINT_DTYPE, default_context

INT_MAX = 2 ** 31 - 1


def _kp(a):
    return np.ascontiguousarray(a, KEYPOINT_DTYPE)


def _u8(a):
    return np.ascontiguousarray(a, np.uint8)


def _i32(a):
    return np.ascontiguousarray(a, np.int32)


def _pp(a):
    return ptr(a) if a.size else None


def window_search(info, kps2, desc2, kps1, desc1, mp1, window: int, min_level: int, max_level: int = INT_MAX,
                  nnratio: float = 0.9, check_ori: bool = True, ctx=None):
    """ORBmatcher(nnratio, check_ori).WindowSearch(F1, F2, window, out,
    min_level, max_level) (ORBmatcher.cc:979-1086) -> (nmatches, out[n2])."""
    ctx = ctx or default_context()
    k2, d2, k1, d1, m1 = _kp(kps2), _u8(desc2), _kp(kps1), _u8(desc1), _i32(mp1)
    out = np.full(max(len(k2), 1), -1, np.int32)
    nm = ctypes.c_int()
    check(lib().gf_window_search(ctx.handle, ctypes.byref(info), _pp(k2), _pp(d2), len(k2), _pp(k1), _pp(d1), _pp(m1),
                                 len(k1), int(window), int(min_level), int(max_level), ctypes.c_float(nnratio),
                                 int(check_ori), ptr(out), ctypes.byref(nm)))
    return nm.value, out[:len(k2)].copy()


def search_frames(info, kps2, desc2, Tcw2, kps1, desc1, mp1, pos1, window: int, kp2mp, score, nnratio: float = 0.9,
                  ctx=None):
    """ORBmatcher(nnratio).SearchByProjection(F1, F2, window, matches)
    (ORBmatcher.cc:1089-1168) -> (nmatches, kp2mp, score)."""
    ctx = ctx or default_context()
    k2, d2, k1, d1, m1 = _kp(kps2), _u8(desc2), _kp(kps1), _u8(desc1), _i32(mp1)
    p1 = np.ascontiguousarray(pos1, np.float32)
    T = np.ascontiguousarray(Tcw2, np.float32).reshape(16)
    km, sc = np.array(kp2mp, np.int32), np.array(score, np.int32)
    nm = ctypes.c_int()
    check(lib().gf_search_frames(ctx.handle, ctypes.byref(info), _pp(k2), _pp(d2), len(k2), ptr(T), _pp(k1), _pp(d1),
                                 _pp(m1), _pp(p1), len(k1), int(window), ctypes.c_float(nnratio), _pp(km), _pp(sc),
                                 ctypes.byref(nm)))
    return nm.value, km, sc


def search_kf_projection(info, kps, desc, Tcw, kf_kps, kf_mp, mps, mp_desc, found, th: float, orb_dist: int, kp2mp,
                         score, check_ori: bool = True, ctx=None):
    """ORBmatcher(0.9, check_ori).SearchByProjection(F, pKF, sAlreadyFound,
    th, ORBdist) (ORBmatcher.cc:2204-2336); found = a byte per map point ->
    (nmatches, kp2mp, score)."""
    ctx = ctx or default_context()
    k, d, kk, km_ = _kp(kps), _u8(desc), _kp(kf_kps), _i32(kf_mp)
    m, md, f = np.ascontiguousarray(mps, MAP_POINT_DTYPE), _u8(mp_desc), _u8(found)
    T = np.ascontiguousarray(Tcw, np.float32).reshape(16)
    km, sc = np.array(kp2mp, np.int32), np.array(score, np.int32)
    nm = ctypes.c_int()
    check(lib().gf_search_kf_projection(ctx.handle, ctypes.byref(info), _pp(k), _pp(d), len(k), ptr(T), _pp(kk),
                                        _pp(km_), len(kk), _pp(m), _pp(md), len(m), _pp(f), ctypes.c_float(th),
                                        int(orb_dist), int(check_ori), _pp(km), _pp(sc), ctypes.byref(nm)))
    return nm.value, km, sc


def reloc_candidates(words, values, db, kf_bad, cov_off, cov, query: int, state, ctx=None):
    """KeyFrameDatabase::DetectRelocalisationCandidates for a BowVector against
    a pipeline.KeyframeDB; state (RELOC_KF_DTYPE, db.nkf entries) is updated
    in place as the keyframes' fields are -> candidate keyframes in order."""
    ctx = ctx or default_context()
    w, v = _i32(words), np.ascontiguousarray(values, np.float64)
    kb = None if kf_bad is None else _u8(kf_bad)
    co, cv = _i32(cov_off), _i32(cov)
    st = np.ascontiguousarray(state[:db.nkf])
    out = np.zeros(64, np.int32)
    nc = ctypes.c_int()
    check(lib().gf_reloc_candidates(ctx.handle, _pp(w), _pp(v), len(w), ctypes.byref(db.struct()),
                                    None if kb is None else _pp(kb), ptr(co), _pp(cv), ctypes.c_uint32(query),
                                    _pp(st), ptr(out), ctypes.byref(nc)))
    state[:db.nkf] = st
    return out[:nc.value].copy()
