"""Host-side mirror of ORB_SLAM::Observability (include/Observability.h) over
libgfslam: PWLS kinematics (host, as in the reference), per-landmark
Jacobian/information blocks, log-det, active map matching and max-volume
subset selection (GPU)."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr
from .matcher import MP_VIEW_DTYPE, Frame
from .orb import default_context


class ObsCamera(ctypes.Structure):
    _fields_ = [("fu", ctypes.c_double), ("fv", ctypes.c_double), ("cx", ctypes.c_double), ("cy", ctypes.c_double),
                ("nrows", ctypes.c_int32), ("ncols", ctypes.c_int32), ("min_x", ctypes.c_int32),
                ("max_x", ctypes.c_int32), ("min_y", ctypes.c_int32), ("max_y", ctypes.c_int32),
                ("bound_x", ctypes.c_int32), ("bound_y", ctypes.c_int32), ("bound_depth", ctypes.c_float)]

    @classmethod
    def from_focal(cls, f, nrows, ncols, cx, cy, dx, dy, bound=20, bound_depth=0.0):
        """Observability(f, nRows, nCols, Cx, Cy, k1, k2, dx, dy): fu = f/dx."""
        return cls(f / dx, f / dy, cx, cy, int(nrows), int(ncols), 0, int(ncols), 0, int(nrows), bound, bound,
                   bound_depth)

    @classmethod
    def from_intrinsics(cls, fu, fv, cx, cy, ncols, nrows, bound=20, bound_depth=0.0, bound_y=None):
        by = bound if bound_y is None else bound_y
        return cls(fu, fv, cx, cy, int(nrows), int(ncols), 0, int(ncols), 0, int(nrows), bound, by, bound_depth)

    @classmethod
    def for_tracking(cls, fu, fv, cx, cy, ncols, nrows):
        """The margins Tracking sets: mBoundX/YInFrame = 0.1 * image extent
        (int), mBoundDepth = 0 (Tracking.cc:875-877)."""
        return cls.from_intrinsics(fu, fv, cx, cy, ncols, nrows, bound=int(0.1 * ncols), bound_y=int(0.1 * nrows))


class Kine(ctypes.Structure):
    """gf_kine (KineStruct, Util.hpp:170-177)."""

    _fields_ = [("dt", ctypes.c_double), ("dt_inseg", ctypes.c_double), ("Xv", ctypes.c_double * 13),
                ("F_Q", ctypes.c_double * 16), ("F_Omg", ctypes.c_double * 12), ("F_Q_inSeg", ctypes.c_double * 16),
                ("F_Omg_inSeg", ctypes.c_double * 12), ("Tcw", ctypes.c_float * 16)]


class Rng(ctypes.Structure):
    """gf_rng: glibc rand() state (std::srand / std::rand)."""

    _fields_ = [("state", ctypes.c_int32 * 31), ("f", ctypes.c_int32), ("r", ctypes.c_int32)]

    @classmethod
    def seeded(cls, seed: int = 1):
        r = cls()
        check(lib().gf_rng_seed(ctypes.byref(r), ctypes.c_uint32(seed)))
        return r

    def next(self, n: int) -> np.ndarray:
        out = np.zeros(n, np.int32)
        check(lib().gf_rng_next(ctypes.byref(self), ptr(out), n))
        return out


class Observability:
    def __init__(self, camera: ObsCamera, ctx=None):
        self.camera = camera
        self.ctx = ctx or default_context()
        self.Xv = np.zeros(13)
        self.kinematic: list[Kine] = []
        self.rng = Rng.seeded(1)

    # ---------------------------------------------------------- kinematics (host)
    def updatePWLSVec(self, time_prev, Tcw_prev, time_cur, Twc_cur):
        xv = np.zeros(13)
        check(lib().gf_obs_update(ctypes.c_double(time_prev), ptr(np.ascontiguousarray(Tcw_prev, np.float32)),
                                  ctypes.c_double(time_cur), ptr(np.ascontiguousarray(Twc_cur, np.float32)),
                                  ptr(xv)))
        self.Xv = xv

    def predictPWLSVec(self, dt, num_seg_pred):
        out = (Kine * num_seg_pred)()
        check(lib().gf_obs_predict(ptr(np.ascontiguousarray(self.Xv, np.float64)), ctypes.c_double(dt),
                                   int(num_seg_pred), out))
        self.kinematic = list(out)

    # ---------------------------------------------------------- matrices (GPU)
    def build_info(self, pos, sigma2=None, check_viz=False, kine_idx=0):
        """batchInfoMat_Map (sigma2=None) / batchInfoMat_Frame (per-landmark sigma^2)."""
        pos = np.ascontiguousarray(pos, np.float32).reshape(-1, 3)
        n = len(pos)
        H = np.zeros((n, 14))
        info = np.zeros((n, 49))
        uv = np.zeros((n, 2), np.float32)
        valid = np.zeros(n, np.uint8)
        s2 = None if sigma2 is None else np.ascontiguousarray(sigma2, np.float32)
        xv = np.array(self.kinematic[kine_idx].Xv[:], np.float64)
        check(lib().gf_obs_build_info(self.ctx.handle, ctypes.byref(self.camera), ptr(xv), ptr(pos), ptr(s2), n,
                                      int(check_viz), ptr(H), ptr(info), ptr(uv), ptr(valid)))
        return H, info, uv, valid

    def logDet(self, M) -> np.ndarray:
        M = np.ascontiguousarray(M, np.float64).reshape(-1, 49)
        out = np.zeros(len(M))
        check(lib().gf_logdet(self.ctx.handle, ptr(M), len(M), ptr(out)))
        return out

    def runActiveMapMatching(self, F: Frame, views, mp_desc, updated, info, H, uv, base, num_to_match,
                             th=1.0, nnratio=0.8):
        views = np.ascontiguousarray(views, MP_VIEW_DTYPE)
        m = len(views)
        left = np.zeros(max(m, 1), np.int32)
        nleft, nmatched = ctypes.c_int(), ctypes.c_int()
        sigma2 = (F.info.scale_factors().astype(np.float32) ** 2).astype(np.float32)
        check(lib().gf_obs_active_match(
            self.ctx.handle, ctypes.byref(F.info), ptr(F.mvKeysUn), ptr(F.mDescriptors), F.N, ptr(views),
            ptr(np.ascontiguousarray(mp_desc, np.uint8)), ptr(np.ascontiguousarray(updated, np.uint8)),
            ptr(np.ascontiguousarray(info, np.float64)), ptr(np.ascontiguousarray(H, np.float64)),
            ptr(np.ascontiguousarray(uv, np.float32)), m, ptr(np.ascontiguousarray(base, np.float64)), ptr(sigma2),
            int(num_to_match), ctypes.c_float(th), ctypes.c_float(nnratio), ctypes.byref(self.rng),
            ptr(F.mvpMapPoints), ptr(F.mvpMatchScore), ptr(left), ctypes.byref(nleft), ctypes.byref(nmatched)))
        self.mLeftMapPoints = left[:nleft.value].copy()
        return nmatched.value

    def setSelction_Number(self, num_good_inlier: int, greedy_mtd: int, map_pos, max_threads: int = 8):
        """Observability::setSelction_Number over map points
        (Observability.cc:1021-1247) at kinematic[1] (mKineIdx = 1): the
        selected map indices (mpVec idx) in selection order."""
        pos = np.ascontiguousarray(map_pos, np.float32).reshape(-1, 3)
        xv = np.ascontiguousarray(self.kinematic[1].Xv[:] if len(self.kinematic) > 1 else self.Xv, np.float64)
        out = np.zeros(max(len(pos), 1), np.int32)
        nout = ctypes.c_int()
        check(lib().gf_select_map_points(self.ctx.handle, ctypes.byref(self.camera), ptr(xv), ptr(pos), len(pos),
                                         int(num_good_inlier), int(greedy_mtd), int(max_threads),
                                         ctypes.byref(self.rng), ptr(out), ctypes.byref(nout)))
        return out[:nout.value].copy()

    def maxvol_select(self, info, score, k, sample_scale, mode):
        info = np.ascontiguousarray(info, np.float64).reshape(-1, 49)
        n = len(info)
        out = np.zeros(max(n, 1), np.int32)
        nout = ctypes.c_int()
        check(lib().gf_maxvol_select(self.ctx.handle, ptr(info), ptr(np.ascontiguousarray(score, np.float64)), n,
                                     int(k), ctypes.c_double(sample_scale), int(mode), ctypes.byref(self.rng),
                                     ptr(out), ctypes.byref(nout)))
        return out[:nout.value].copy()
