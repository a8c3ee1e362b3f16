"""Monocular map initialisation: the reference's ``ORB_SLAM::Initializer``
(include/Initializer.h, src/Initializer.cc) on the device, behind
``gf_initialize`` / ``gf_initialize_dev`` (include/gfslam/abi.h).

``Initializer`` keeps the reference's interface: built from the reference
frame's undistorted keypoints, the calibration, sigma and the RANSAC
iteration count (ctor, Initializer.cc:31-42); ``initialize(current_keys,
matches12, rng)`` is ``Initialize`` (:44-132) and returns ``(ok, R21, t21,
vP3D, vbTriangulated)`` like the reference's out-parameters. The 8-point sets
come from the process-wide ``std::rand()`` (:87), here a :class:`Rand` the
caller passes. ``last_result`` holds the full :data:`INIT_RESULT_DTYPE`
record (scores, kept models, nGood per hypothesis, parallax).
"""
from __future__ import annotations

import numpy as np

from ._lib import check, lib, ptr
from .matcher import default_context
from .orb import KEYPOINT_DTYPE
from .pnp import Rand

INIT_RESULT_DTYPE = np.dtype([("ok", "i4"), ("model", "i4"), ("nmatches", "i4"), ("iter_H", "i4"),
                              ("iter_F", "i4"), ("ninliers_H", "i4"), ("ninliers_F", "i4"), ("best", "i4"),
                              ("ngood", "i4", (8,)), ("SH", "f4"), ("SF", "f4"), ("RH", "f4"),
                              ("parallax", "f4"), ("H21", "f4", (9,)), ("F21", "f4", (9,)), ("R21", "f4", (9,)),
                              ("t21", "f4", (3,))])
assert INIT_RESULT_DTYPE.itemsize == 200

# THRES_INIT_MPT_NUM / 2 (include/Initializer.h, INIT_WITH_MOTION_PRIOR off)
MIN_TRIANGULATED = 50

__all__ = ["Initializer", "INIT_RESULT_DTYPE", "MIN_TRIANGULATED", "Rand"]


class Initializer:
    def __init__(self, reference_keys_un, K, sigma: float = 1.0, iterations: int = 200,
                 min_triangulated: int = MIN_TRIANGULATED, ctx=None):
        self.ctx = ctx or default_context()
        self.keys1 = np.ascontiguousarray(reference_keys_un, KEYPOINT_DTYPE)
        self.K = np.ascontiguousarray(np.asarray(K, np.float32).reshape(9))
        self.sigma = float(sigma)
        self.iterations = int(iterations)
        self.min_triangulated = int(min_triangulated)
        self.last_result = np.zeros(1, INIT_RESULT_DTYPE)

    def initialize(self, current_keys_un, matches12, rng: Rand):
        keys2 = np.ascontiguousarray(current_keys_un, KEYPOINT_DTYPE)
        m = np.ascontiguousarray(matches12, np.int32)
        n1 = len(self.keys1)
        if len(m) != n1:
            raise ValueError("matches12 needs one entry per reference keypoint")
        res = np.zeros(1, INIT_RESULT_DTYPE)
        p3d = np.zeros((n1, 3), np.float32)
        tri = np.zeros(n1, np.uint8)
        check(lib().gf_initialize(self.ctx.handle, ptr(self.K), self.sigma, self.iterations, self.min_triangulated,
                                  ptr(self.keys1), n1, ptr(keys2), len(keys2), ptr(m), ptr(rng.state), ptr(res),
                                  ptr(p3d), ptr(tri)))
        self.last_result = res
        r = res[0]
        ok = bool(r["ok"])
        R21 = r["R21"].reshape(3, 3).copy() if ok else None
        t21 = r["t21"].reshape(3, 1).copy() if ok else None
        return ok, R21, t21, p3d, tri.astype(bool)


def initialize_device(ctx, K, kps1, kps2, matches12, rng_state, sigma: float = 1.0, iterations: int = 200,
                      min_triangulated: int = MIN_TRIANGULATED, stream=None):
    """Device family: torch tensors on the GPU (kps as raw KEYPOINT_DTYPE bytes,
    [n, 28] uint8; matches12 int32; rng_state [132] uint8). Returns
    (result bytes [200] uint8, p3d [n1, 3] f32, triangulated [n1] u8), all on
    the device; rng_state advances in place."""
    import torch

    n1, n2 = kps1.shape[0], kps2.shape[0]
    dev = kps1.device
    res = torch.zeros(INIT_RESULT_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    p3d = torch.zeros((n1, 3), dtype=torch.float32, device=dev)
    tri = torch.zeros(n1, dtype=torch.uint8, device=dev)
    Kf = np.ascontiguousarray(np.asarray(K, np.float32).reshape(9))
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    check(lib().gf_initialize_dev(ctx.handle, ptr(Kf), float(sigma), int(iterations), int(min_triangulated),
                                  kps1.data_ptr(), n1, kps2.data_ptr(), n2, matches12.data_ptr(),
                                  rng_state.data_ptr(), res.data_ptr(), p3d.data_ptr(), tri.data_ptr(), s))
    return res, p3d, tri


def initialize_batch_device(ctx, K, kps1, n1, kps2, n2, matches12, rng_states, sigma: float = 1.0,
                            iterations: int = 200, min_triangulated: int = MIN_TRIANGULATED, stream=None):
    """Device batch (gf_initialize_batch_dev): kps1 [P, cap1, 28] / kps2
    [P, cap2, 28] uint8 (KEYPOINT_DTYPE rows), n1 / n2 [P] int32, matches12
    [P, cap1] int32, rng_states [P, 132] uint8 (advanced in place). Returns
    (results [P, 200] uint8, p3d [P, cap1, 3] f32, triangulated [P, cap1] u8)."""
    import torch

    P, cap1 = kps1.shape[0], kps1.shape[1]
    cap2 = kps2.shape[1]
    dev = kps1.device
    res = torch.zeros((P, INIT_RESULT_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    p3d = torch.zeros((P, cap1, 3), dtype=torch.float32, device=dev)
    tri = torch.zeros((P, cap1), dtype=torch.uint8, device=dev)
    Kf = np.ascontiguousarray(np.asarray(K, np.float32).reshape(9))
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    check(lib().gf_initialize_batch_dev(ctx.handle, P, ptr(Kf), float(sigma), int(iterations), int(min_triangulated),
                                        kps1.data_ptr(), cap1, n1.data_ptr(), kps2.data_ptr(), cap2, n2.data_ptr(),
                                        matches12.data_ptr(), rng_states.data_ptr(), res.data_ptr(), p3d.data_ptr(),
                                        tri.data_ptr(), s))
    return res, p3d, tri
