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
