"""Relocalisation PnP: the reference's ``ORB_SLAM::PnPsolver``
(include/PnPsolver.h, src/PnPsolver.cc) on the device, EPnP minimal sets in
RANSAC plus the inlier refinement, behind ``gf_pnp_init`` /
``gf_pnp_iterate`` / ``gf_pnp_iterate_dev`` (include/gfslam/abi.h).

``PnPsolver`` keeps the reference's interface: built from a frame's matched
map points (ctor :39-82, bad points skipped), ``set_ransac_parameters``
(:93-129), ``iterate(n)`` (:137-230) returning ``(Tcw or None, no_more,
inliers, n_inliers)`` with ``inliers`` indexed by keypoint like the
reference's ``vbInliers``, and ``find()`` (:131-135). The process-wide
``std::rand()`` of the reference is a :class:`Rand` the caller shares between
solvers (Tracking::Relocalization interleaves them, Tracking.cc:3930-3945).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr
from .matcher import default_context

PNP_PARAMS_DTYPE = np.dtype([("probability", "f8"), ("min_inliers", "i4"), ("max_iterations", "i4"),
                             ("min_set", "i4"), ("epsilon", "f4"), ("th2", "f4")], align=True)
PNP_STATE_DTYPE = np.dtype([("n", "i4"), ("min_inliers", "i4"), ("max_iterations", "i4"), ("min_set", "i4"),
                            ("epsilon", "f4"), ("th2", "f4"), ("iterations", "i4"), ("best_inliers", "i4"),
                            ("best_Tcw", "f4", (16,))], align=True)
RNG_DTYPE = np.dtype([("state", "i4", (31,)), ("f", "i4"), ("r", "i4")])
GF_PNP_FOUND, GF_PNP_NOMORE, GF_PNP_REFINED = 1, 2, 4

assert PNP_PARAMS_DTYPE.itemsize == 32 and PNP_STATE_DTYPE.itemsize == 96 and RNG_DTYPE.itemsize == 132


def pnp_params(probability=0.99, min_inliers=8, max_iterations=300, min_set=4, epsilon=0.4, th2=5.991):
    """SetRansacParameters arguments; the defaults are PnPsolver.h's."""
    p = np.zeros(1, PNP_PARAMS_DTYPE)
    p[0] = (probability, min_inliers, max_iterations, min_set, epsilon, th2)
    return p


class Rand:
    """The glibc ``std::rand()`` state (``gf_rng``), seeded like ``std::srand``."""

    def __init__(self, seed: int = 1):
        self.state = np.zeros(1, RNG_DTYPE)
        check(lib().gf_rng_seed(ptr(self.state), ctypes.c_uint32(seed)))


class PnPsolver:
    def __init__(self, keypoints_un, map_point_pos, level_sigma2, K, bad=None, ctx=None):
        """keypoints_un: the frame's mvKeysUn (KEYPOINT_DTYPE); map_point_pos:
        [n_kps, 3] world positions with NaN rows where vpMapPointMatches[i] is
        NULL; bad: optional per-keypoint isBad() flags; K = (fx, fy, cx, cy)."""
        self.ctx = ctx or default_context()
        pos = np.asarray(map_point_pos, np.float32).reshape(-1, 3)
        keep = ~np.isnan(pos).any(axis=1)
        if bad is not None:
            keep &= ~np.asarray(bad, bool)
        self.n_kps = len(pos)
        self.kp_idx = np.nonzero(keep)[0].astype(np.int32)        # mvKeyPointIndices
        self.p3d = np.ascontiguousarray(pos[keep])
        kps = keypoints_un[self.kp_idx]
        self.p2d = np.ascontiguousarray(np.stack([kps["x"], kps["y"]], 1), np.float32)
        self.sigma2 = np.ascontiguousarray(np.asarray(level_sigma2, np.float32)[kps["octave"]])
        self.K = np.asarray(K, np.float32).reshape(4)
        self.best_mask = np.zeros(max(len(self.p3d), 1), np.uint8)
        self.set_ransac_parameters()

    @property
    def N(self) -> int:
        return len(self.p3d)

    def set_ransac_parameters(self, probability=0.99, min_inliers=8, max_iterations=300, min_set=4, epsilon=0.4,
                              th2=5.991):
        # SetRansacParameters (PnPsolver.cc:93-129) leaves mnIterations,
        # mnBestInliers and the best pose as they are: keep them across a re-call
        old = getattr(self, "state", None)
        self.state = np.zeros(1, PNP_STATE_DTYPE)
        prm = pnp_params(probability, min_inliers, max_iterations, min_set, epsilon, th2)
        check(lib().gf_pnp_init(self.N, ptr(prm), ptr(self.state)))
        if old is not None:
            for k in ("iterations", "best_inliers", "best_Tcw"):
                self.state[k] = old[k]

    def iterate(self, n_iterations: int, rng: Rand):
        T = np.zeros(16, np.float32)
        inl = np.zeros(max(self.N, 1), np.uint8)
        ninl = np.zeros(1, np.int32)
        fl = np.zeros(1, np.int32)
        check(lib().gf_pnp_iterate(self.ctx.handle, ptr(self.p3d), ptr(self.p2d), ptr(self.sigma2), ptr(self.K),
                                   ptr(self.state), ptr(self.best_mask), int(n_iterations), ptr(rng.state), ptr(T),
                                   ptr(inl), ptr(ninl), ptr(fl)))
        vb = np.zeros(self.n_kps, bool)
        vb[self.kp_idx[inl[:self.N].astype(bool)]] = True
        Tcw = T.reshape(4, 4) if fl[0] & GF_PNP_FOUND else None
        return Tcw, bool(fl[0] & GF_PNP_NOMORE), vb, int(ninl[0])

    def find(self, rng: Rand):
        return self.iterate(int(self.state["max_iterations"][0]), rng)
