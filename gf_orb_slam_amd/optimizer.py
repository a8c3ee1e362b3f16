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
