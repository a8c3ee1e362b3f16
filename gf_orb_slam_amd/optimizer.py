"""Host-side mirror of ORB_SLAM::Optimizer::PoseOptimization (include/Optimizer.h:53,
src/Optimizer.cc:279-413) over libgfslam's C-ABI. The LM runs on the GPU
(csrc/poseopt.hip); this module only packs the Frame's matched keypoints into
edges and writes the results back, as the reference does.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr
from .orb import default_context

POSE_EDGE_DTYPE = np.dtype([("X", "<f4", 3), ("z", "<f4", 2), ("inv_sigma2", "<f4")])
assert POSE_EDGE_DTYPE.itemsize == 24


def inv_level_sigma2(nlevels: int = 8, scale_factor: float = 1.2) -> np.ndarray:
    """Frame::mvInvLevelSigma2 = 1 / (scale^level)^2 in float (ORBextractor.cc:443-452)."""
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(s[-1] * np.float32(scale_factor)))
    s = np.array(s, np.float32)
    return (np.float32(1.0) / (s * s)).astype(np.float32)


class Optimizer:
    @staticmethod
    def PoseOptimization(pFrame, map_pos: np.ndarray | None = None, ctx=None) -> int:
        """Motion-only BA of pFrame.mTcw against its matched map points.

        Edges are the keypoints with mvpMapPoints[i] >= 0, in keypoint order.
        Map-point world positions come from map_pos[mvpMapPoints[i]] when given,
        else from pFrame.mp_pos[i]. Updates pFrame.mTcw and pFrame.mvbOutlier
        (matched keypoints only) and returns the number of inliers.
        """
        ctx = ctx or default_context()
        idx = np.nonzero(pFrame.mvpMapPoints >= 0)[0]
        n = len(idx)
        edges = np.zeros(max(n, 1), POSE_EDGE_DTYPE)
        if n:
            mp = pFrame.mvpMapPoints[idx]
            edges["X"][:n] = (np.asarray(map_pos, np.float32)[mp] if map_pos is not None else pFrame.mp_pos[idx])
            kps = pFrame.mvKeysUn[idx]
            edges["z"][:n, 0] = kps["x"]
            edges["z"][:n, 1] = kps["y"]
            invs = inv_level_sigma2(pFrame.info.nlevels, pFrame.info.scale_factor)
            edges["inv_sigma2"][:n] = invs[kps["octave"]]
        Tin = np.ascontiguousarray(pFrame.mTcw, np.float32)
        Tout = np.zeros((4, 4), np.float32)
        outl = np.zeros(max(n, 1), np.uint8)
        ninl = ctypes.c_int32()
        fi = pFrame.info
        check(lib().gf_pose_opt(ctx.handle, ptr(Tin), ptr(edges), n, ctypes.c_float(fi.fx), ctypes.c_float(fi.fy),
                                ctypes.c_float(fi.cx), ctypes.c_float(fi.cy), ptr(Tout), ptr(outl),
                                ctypes.byref(ninl), None))
        pFrame.mTcw = Tout
        if n:
            pFrame.mvbOutlier[idx] = outl[:n]
        return int(ninl.value)

    @staticmethod
    def pose_opt_edges(Tcw, edges: np.ndarray, fx, fy, cx, cy, ctx=None):
        """Raw edge-list form: returns (Tcw_out, outlier[n], ninliers, iterations)."""
        ctx = ctx or default_context()
        edges = np.ascontiguousarray(edges, POSE_EDGE_DTYPE)
        n = len(edges)
        Tin = np.ascontiguousarray(Tcw, np.float32).reshape(4, 4)
        Tout = np.zeros((4, 4), np.float32)
        outl = np.zeros(max(n, 1), np.uint8)
        ninl, iters = ctypes.c_int32(), ctypes.c_int32()
        check(lib().gf_pose_opt(ctx.handle, ptr(Tin), ptr(edges) if n else None, n, ctypes.c_float(fx),
                                ctypes.c_float(fy), ctypes.c_float(cx), ctypes.c_float(cy), ptr(Tout), ptr(outl),
                                ctypes.byref(ninl), ctypes.byref(iters)))
        return Tout, outl[:n].copy(), int(ninl.value), int(iters.value)

    @staticmethod
    def pose_opt_batch_dev(d_Tcw, d_edges, d_nedges, edge_stride: int, fx, fy, cx, cy, d_outlier, d_ninliers,
                           d_iterations=None, ctx=None, stream=None) -> None:
        """Batched device form: torch tensors (or raw pointers) already on the GPU."""
        ctx = ctx or default_context()
        nprob = int(d_nedges.numel()) if hasattr(d_nedges, "numel") else int(len(d_nedges))
        check(lib().gf_pose_opt_batch_dev(ctx.handle, nprob, ptr(d_Tcw), ptr(d_edges), ptr(d_nedges),
                                          int(edge_stride), ctypes.c_float(fx), ctypes.c_float(fy),
                                          ctypes.c_float(cx), ctypes.c_float(cy), ptr(d_outlier), ptr(d_ninliers),
                                          ptr(d_iterations), stream if stream is not None else ctx.stream))


# ---------------------------------------------------------------- local BA (B1)
BA_LOCAL, BA_LOCAL_FIXED, BA_FIXED = 0, 1, 2


class BAProblem(ctypes.Structure):
    """gf_ba_problem (include/gfslam/abi.h): the graph LocalBundleAdjustment builds."""

    _fields_ = [("nkf", ctypes.c_int32), ("npts", ctypes.c_int32), ("nedges", ctypes.c_int32),
                ("kf_Tcw", ctypes.c_void_p), ("kf_kind", ctypes.c_void_p), ("kf_cam", ctypes.c_void_p),
                ("pt_pos", ctypes.c_void_p), ("edge_pt", ctypes.c_void_p), ("edge_kf", ctypes.c_void_p),
                ("edge_z", ctypes.c_void_p), ("edge_inv_sigma2", ctypes.c_void_p)]


class BAResult(ctypes.Structure):
    _fields_ = [("kf_Tcw", ctypes.c_void_p), ("pt_pos", ctypes.c_void_p), ("edge_outlier", ctypes.c_void_p),
                ("iterations", ctypes.c_int32 * 2)]


_BA_FIELDS = (("kf_Tcw", np.float32), ("kf_kind", np.uint8), ("kf_cam", np.float32), ("pt_pos", np.float32),
              ("edge_pt", np.int32), ("edge_kf", np.int32), ("edge_z", np.float32),
              ("edge_inv_sigma2", np.float32))


class BAArrays:
    """Keeps the numpy arrays of one problem alive next to its ctypes views."""

    def __init__(self, prob: dict):
        self.a = {k: np.ascontiguousarray(prob[k], dt) for k, dt in _BA_FIELDS}
        self.nkf, self.npts, self.nedges = len(self.a["kf_kind"]), len(self.a["pt_pos"]), len(self.a["edge_pt"])
        self.problem = BAProblem(self.nkf, self.npts, self.nedges,
                                 *[self.a[k].ctypes.data if self.a[k].size else None for k, _ in _BA_FIELDS])
        self.kf_Tcw = np.zeros((self.nkf, 4, 4), np.float32)
        self.pt_pos = np.zeros((self.npts, 3), np.float32)
        self.outlier = np.zeros(max(self.nedges, 1), np.uint8)
        self.result = BAResult(self.kf_Tcw.ctypes.data, self.pt_pos.ctypes.data, self.outlier.ctypes.data)

    def out(self):
        """(kf_Tcw [nkf,4,4], pt_pos [npts,3], edge_outlier [nedges], iterations (it5, it10))."""
        return (self.kf_Tcw.copy(), self.pt_pos.copy(), self.outlier[:self.nedges].copy(),
                tuple(int(i) for i in self.result.iterations))


def local_bundle_adjustment(prob: dict, ctx=None, stop_flag=None):
    """Optimizer::LocalBundleAdjustment(pKF, pbStopFlag) (Optimizer.cc:1515-1764)
    on one local window (dict with the gf_ba_problem arrays, e.g.
    synth.synth_lba_problem). stop_flag: optional ctypes.c_uint8 polled as
    mbAbortBA. Returns (kf_Tcw, pt_pos, edge_outlier, iterations)."""
    ctx = ctx or default_context()
    arr = BAArrays(prob)
    check(lib().gf_local_ba_stop(ctx.handle, ctypes.byref(arr.problem), ctypes.byref(arr.result),
                                 ctypes.byref(stop_flag) if stop_flag is not None else None))
    return arr.out()


class LocalBAPlan:
    """Batched device path: nprob local windows uploaded once, solved together
    (gf_ba_plan_create / _solve / _results)."""

    def __init__(self, probs: list, ctx=None):
        self.ctx = ctx or default_context()
        self.arrs = [BAArrays(p) for p in probs]
        ps = (BAProblem * len(probs))(*[a.problem for a in self.arrs])
        self.handle = ctypes.c_void_p()
        check(lib().gf_ba_plan_create(self.ctx.handle, len(probs), ps, ctypes.byref(self.handle)))

    def solve(self, stream=None) -> int:
        steps = ctypes.c_int()
        check(lib().gf_ba_plan_solve(self.handle, stream if stream is not None else self.ctx.stream,
                                     ctypes.byref(steps)))
        return steps.value

    def results(self) -> list:
        rs = (BAResult * len(self.arrs))(*[a.result for a in self.arrs])
        check(lib().gf_ba_plan_results(self.handle, rs))
        for a, r in zip(self.arrs, rs):
            a.result.iterations[:] = r.iterations[:]
        return [a.out() for a in self.arrs]

    def close(self) -> None:
        if self.handle:
            lib().gf_ba_plan_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
