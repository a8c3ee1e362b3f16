"""Host-side mirror of ORB_SLAM::ORBmatcher / Frame (include/ORBmatcher.h,
include/Frame.h) over libgfslam's C-ABI.

Frame-to-map associations are index arrays instead of pointers:
`Frame.mvpMapPoints[i]` is the map-point id matched to keypoint i (-1 for
NULL), `Frame.mvpMatchScore[i]` its Hamming distance (999 when unmatched,
Frame.cc:66). All matching runs on the GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr
from .orb import KEYPOINT_DTYPE, default_context

MAP_POINT_DTYPE = np.dtype([("pos", "<f4", 3), ("normal", "<f4", 3), ("min_dist", "<f4"), ("max_dist", "<f4")])
FUSE_RESULT_DTYPE = np.dtype([("kp", "<i4"), ("action", "<i4"), ("target", "<i4")])
FUSE_NONE, FUSE_ADD, FUSE_REPLACE, FUSE_KEEP = 0, 1, 2, 3
MP_VIEW_DTYPE = np.dtype([("u", "<f4"), ("v", "<f4"), ("view_cos", "<f4"), ("level", "<i4"), ("in_view", "<i4")])
assert MAP_POINT_DTYPE.itemsize == 32 and MP_VIEW_DTYPE.itemsize == 20


class FrameInfo(ctypes.Structure):
    """gf_frame_info: image bounds, intrinsics and scale pyramid of a Frame."""

    _fields_ = [("min_x", ctypes.c_int32), ("max_x", ctypes.c_int32), ("min_y", ctypes.c_int32),
                ("max_y", ctypes.c_int32), ("fx", ctypes.c_float), ("fy", ctypes.c_float), ("cx", ctypes.c_float),
                ("cy", ctypes.c_float), ("nlevels", ctypes.c_int32), ("scale_factor", ctypes.c_float)]

    @classmethod
    def make(cls, width, height, fx, fy, cx, cy, nlevels=8, scale_factor=1.2):
        # undistortion bypassed (k1 == 0): bounds are the image (Frame.cc:470-476)
        return cls(0, int(width), 0, int(height), fx, fy, cx, cy, nlevels, scale_factor)

    def scale_factors(self) -> np.ndarray:
        s = [np.float32(1.0)]
        for _ in range(1, self.nlevels):
            s.append(np.float32(s[-1] * np.float32(self.scale_factor)))
        return np.array(s, np.float32)


class FuseProblem(ctypes.Structure):
    """gf_fuse_problem: one (keyframe, candidate list) of gf_fuse_dev; device pointers."""

    _fields_ = [("Tcw", ctypes.c_float * 16), ("Ow", ctypes.c_float * 3), ("kps", ctypes.c_void_p),
                ("desc", ctypes.c_void_p), ("n", ctypes.c_int32), ("kf_mp", ctypes.c_void_p),
                ("kf_mp_bad", ctypes.c_void_p), ("mps", ctypes.c_void_p), ("mp_desc", ctypes.c_void_p),
                ("mp_skip", ctypes.c_void_p), ("mp_ids", ctypes.c_void_p), ("m", ctypes.c_int32),
                ("th", ctypes.c_float), ("res", ctypes.c_void_p), ("nfused", ctypes.c_void_p)]

    @classmethod
    def make(cls, Tcw, Ow, bufs, n, m, th):
        """bufs = device tensors (kps, desc, kf_mp, kf_mp_bad|None, mps, mp_desc,
        mp_skip|None, mp_ids|None, res, nfused)."""
        q = cls()
        q.Tcw[:] = [float(x) for x in np.asarray(Tcw, np.float32).reshape(16)]
        q.Ow[:] = [float(x) for x in np.asarray(Ow, np.float32).reshape(3)]
        p = [None if b is None else b.data_ptr() for b in bufs]
        (q.kps, q.desc, q.kf_mp, q.kf_mp_bad, q.mps, q.mp_desc, q.mp_skip, q.mp_ids, q.res, q.nfused) = p
        q.n, q.m, q.th = n, m, th
        return q


class Frame:
    """Keypoints + descriptors of one image with its association state."""

    def __init__(self, keypoints: np.ndarray, descriptors: np.ndarray, info: FrameInfo,
                 Tcw: np.ndarray | None = None):
        self.mvKeys = self.mvKeysUn = np.ascontiguousarray(keypoints, KEYPOINT_DTYPE)
        self.mDescriptors = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        self.N = len(self.mvKeys)
        self.info = info
        self.mvpMapPoints = np.full(self.N, -1, np.int32)
        self.mvpMatchScore = np.full(self.N, 999, np.int32)
        self.mvbOutlier = np.zeros(self.N, np.uint8)
        self.mTcw = None if Tcw is None else np.ascontiguousarray(Tcw, np.float32).reshape(4, 4)
        self.mp_pos = np.zeros((self.N, 3), np.float32)  # world position of the matched map point

    def isInFrustum(self, map_points: np.ndarray, viewingCosLimit: float = 0.5, ctx=None) -> np.ndarray:
        """Frame::isInFrustum for every map point; returns MP_VIEW_DTYPE[M]."""
        ctx = ctx or default_context()
        mps = np.ascontiguousarray(map_points, MAP_POINT_DTYPE)
        views = np.zeros(len(mps), MP_VIEW_DTYPE)
        n = ctypes.c_int()
        check(lib().gf_frustum(ctx.handle, ctypes.byref(self.info), ptr(self.mTcw), ptr(mps), len(mps),
                               ctypes.c_float(viewingCosLimit), ptr(views), ctypes.byref(n)))
        return views


class ORBmatcher:
    TH_HIGH, TH_LOW, HISTO_LENGTH = 100, 50, 30

    def __init__(self, nnratio: float = 0.6, checkOri: bool = True, ctx=None):
        self.mfNNratio, self.mbCheckOrientation = float(nnratio), bool(checkOri)
        self.ctx = ctx or default_context()

    @staticmethod
    def DescriptorDistance(a: np.ndarray, b: np.ndarray, ctx=None) -> np.ndarray:
        ctx = ctx or default_context()
        a = np.ascontiguousarray(a, np.uint8).reshape(-1, 32)
        b = np.ascontiguousarray(b, np.uint8).reshape(-1, 32)
        out = np.zeros(len(a), np.int32)
        check(lib().gf_descriptor_distance(ctx.handle, ptr(a), ptr(b), len(a), ptr(out)))
        return out

    def SearchByProjection(self, F: Frame, views: np.ndarray, mp_desc: np.ndarray, th: float = 3) -> int:
        """ORBmatcher::SearchByProjection(Frame&, vector<MapPoint*>, th) (ORBmatcher.cc:384)."""
        views = np.ascontiguousarray(views, MP_VIEW_DTYPE)
        mp_desc = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        n = ctypes.c_int()
        check(lib().gf_match_project(self.ctx.handle, ctypes.byref(F.info), ptr(F.mvKeysUn), ptr(F.mDescriptors),
                                     F.N, ptr(views), ptr(mp_desc), len(views), ctypes.c_float(th),
                                     ctypes.c_float(self.mfNNratio), ptr(F.mvpMapPoints), ptr(F.mvpMatchScore),
                                     ctypes.byref(n)))
        return n.value

    def SearchByProjection_Budget(self, F: Frame, views: np.ndarray, mp_desc: np.ndarray, th: float,
                                  time_constr: float, found: np.ndarray | None = None) -> int:
        """ORBmatcher::SearchByProjection_Budget (ORBmatcher.cc:276-379): the
        M2 search with MapPoint::IncreaseFound on every match and a wall-clock
        cap. A non-positive budget matches nothing (:281-282); any positive
        budget runs the whole list (parity mode: the device pass finishes far
        inside the reference's budgets, and a clock cut-off would make the
        result timing-dependent). `found` (per map point, optional) receives
        the IncreaseFound increments."""
        if time_constr <= 0:
            return 0
        before = F.mvpMapPoints.copy()
        n = self.SearchByProjection(F, views, mp_desc, th)
        if found is not None:
            new = F.mvpMapPoints[(F.mvpMapPoints >= 0) & (before < 0)]
            np.add.at(found, new, 1)
        return n

    def Fuse(self, KF: Frame, Ow: np.ndarray | None, map_points: np.ndarray, mp_desc: np.ndarray,
             th: float = 3.0, kf_mp_bad: np.ndarray | None = None, mp_skip: np.ndarray | None = None,
             mp_ids: np.ndarray | None = None):
        """ORBmatcher::Fuse(KeyFrame*, vector<MapPoint*>&, th) (ORBmatcher.cc:1590-1707).

        KF: the keyframe as a Frame (mvpMapPoints = ids at its slots, mTcw its
        pose); Ow its camera centre (default -Rcw^T tcw). Returns (nFused,
        FUSE_RESULT_DTYPE[m]): per candidate the fused keypoint and the action
        the reference takes there (FUSE_ADD / FUSE_REPLACE into `target` /
        FUSE_KEEP). The keyframe's slots are updated for FUSE_ADD."""
        mps = np.ascontiguousarray(map_points, MAP_POINT_DTYPE)
        md = np.ascontiguousarray(mp_desc, np.uint8).reshape(-1, 32)
        if Ow is None:
            Ow = camera_center(KF.mTcw)
        Ow = np.ascontiguousarray(Ow, np.float32).reshape(3)
        res = np.zeros(len(mps), FUSE_RESULT_DTYPE)
        opt = lambda a, dt: None if a is None else np.ascontiguousarray(a, dt)
        bad, skip, ids = opt(kf_mp_bad, np.uint8), opt(mp_skip, np.uint8), opt(mp_ids, np.int32)
        n = ctypes.c_int()
        check(lib().gf_fuse(self.ctx.handle, ctypes.byref(KF.info), ptr(KF.mTcw), ptr(Ow), ptr(KF.mvKeysUn),
                            ptr(KF.mDescriptors), KF.N, ptr(KF.mvpMapPoints), ptr(bad), ptr(mps), ptr(md), ptr(skip),
                            ptr(ids), len(mps), ctypes.c_float(th), ptr(res), ctypes.byref(n)))
        add = res["action"] == FUSE_ADD
        KF.mvpMapPoints[res["kp"][add]] = (np.arange(len(mps), dtype=np.int32) if ids is None else ids)[add]
        return n.value, res

    def SearchForTriangulation(self, KF1: tuple, KF2: tuple, F12: np.ndarray, sigma2_2: np.ndarray):
        """ORBmatcher::SearchForTriangulation (ORBmatcher.cc:1426-1588); KF1,
        KF2 = (FeatureVector, descriptors, keypoints, map point per feature).
        Returns (nmatches, vMatches12[n1], vMatchedPairs as (i1, i2) rows)."""
        from .bow import _side
        keep = []
        sa, sb = _side(*KF1, keep), _side(*KF2, keep)
        F = np.ascontiguousarray(F12, np.float32).reshape(9)
        s2 = np.ascontiguousarray(sigma2_2, np.float32)
        out = np.full(max(sa.n, 1), -1, np.int32)
        nm = ctypes.c_int()
        check(lib().gf_search_for_triangulation(self.ctx.handle, int(self.mbCheckOrientation), ctypes.byref(sa),
                                                ctypes.byref(sb), ptr(F), ptr(s2), len(s2), ptr(out),
                                                ctypes.byref(nm)))
        out = out[:sa.n].copy()
        i1 = np.nonzero(out >= 0)[0].astype(np.int32)
        return nm.value, out, np.stack([i1, out[i1]], 1)

    def SearchByProjectionLast(self, CurrentFrame: Frame, LastFrame: Frame, th: float) -> int:
        """ORBmatcher::SearchByProjection(Frame& Cur, const Frame& Last, th) (ORBmatcher.cc:2081)."""
        n = ctypes.c_int()
        check(lib().gf_match_lastframe(self.ctx.handle, ctypes.byref(CurrentFrame.info), ptr(CurrentFrame.mvKeysUn),
                                       ptr(CurrentFrame.mDescriptors), CurrentFrame.N, ptr(CurrentFrame.mTcw),
                                       ptr(LastFrame.mvKeysUn), ptr(LastFrame.mDescriptors),
                                       ptr(LastFrame.mvpMapPoints), ptr(LastFrame.mvbOutlier), ptr(LastFrame.mp_pos),
                                       LastFrame.N, ctypes.c_float(th), int(self.mbCheckOrientation),
                                       ptr(CurrentFrame.mvpMapPoints), ptr(CurrentFrame.mvpMatchScore),
                                       ctypes.byref(n)))
        return n.value


def camera_center(Tcw: np.ndarray) -> np.ndarray:
    """Ow = -Rcw^T tcw in float, as the frustum test computes it."""
    T = np.asarray(Tcw, np.float32).reshape(4, 4)
    out = np.zeros(3, np.float32)
    for c in range(3):
        a, b, d = T[0, c] * T[0, 3], T[1, c] * T[1, 3], T[2, c] * T[2, 3]
        out[c] = -((a + b) + d)
    return out


def compute_distinctive_descriptors(desc: np.ndarray, offsets: np.ndarray, current: np.ndarray | None = None,
                                    ctx=None):
    """MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:197-262) for many
    points: rows offsets[p]..offsets[p+1]-1 of desc observe point p. Returns
    (best row per point relative to offsets[p], -1 when empty; the nmp x 32
    descriptors, `current` kept for empty points)."""
    ctx = ctx or default_context()
    d = np.ascontiguousarray(desc, np.uint8).reshape(-1, 32)
    off = np.ascontiguousarray(offsets, np.int32)
    nmp = len(off) - 1
    best = np.zeros(max(nmp, 1), np.int32)
    out = np.zeros((max(nmp, 1), 32), np.uint8) if current is None else np.ascontiguousarray(current, np.uint8).copy()
    check(lib().gf_distinctive_descriptors(ctx.handle, nmp, ptr(d) if len(d) else None, ptr(off), ptr(best),
                                           ptr(out)))
    return best[:nmp], out[:nmp]


def undistort_keypoints(kps: np.ndarray, K, dist, ctx=None) -> np.ndarray:
    """Frame::UndistortKeyPoints (Frame.cc:389-423): mvKeysUn from mvKeys with
    cv::undistortPoints(K, mDistCoef); a copy when k1 == 0. K = (fx, fy, cx,
    cy); dist = (k1, k2, p1, p2[, k3])."""
    ctx = ctx or default_context()
    k = np.ascontiguousarray(kps, KEYPOINT_DTYPE)
    out = k.copy()
    Kf = np.asarray(K, np.float32).reshape(4)
    d = np.zeros(5, np.float32)
    d[:len(dist)] = np.asarray(dist, np.float32)
    check(lib().gf_undistort_keypoints(ctx.handle, ptr(Kf), ptr(d), ptr(k), len(k), ptr(out)))
    return out
