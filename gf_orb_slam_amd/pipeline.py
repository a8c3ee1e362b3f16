"""Device-resident GF-ORB-SLAM front end for B independent streams on one GPU.

One `step()` runs the per-frame hot path of Tracking::GrabImage for every
stream entirely on the device, through libgfslam's
device-family ABI, with no host round trip:

  ORB extraction (E1-E7)  ->  isInFrustum over the local map (M7)
  ->  SearchByProjection into the local map (M2)

PyTorch only provides device memory and the stream; all compute is in
libgfslam.so.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import synth
from ._lib import check, lib, ptr
from .matcher import MAP_POINT_DTYPE, MP_VIEW_DTYPE, FrameInfo
from .orb import KEYPOINT_DTYPE, Context, ORBextractor


def _torch():
    import torch

    return torch


def build_local_map(kps: np.ndarray, desc: np.ndarray, cam, rng, n_map: int, scale: float = 1.2,
                    nlevels: int = 8, keep: float = 0.9, max_flip: int = 20):
    """Synthetic local map for one frame: most keypoints back-projected at a
    random depth (camera at the origin), descriptor = keypoint descriptor with
    a few flipped bits, plus distractor points with random descriptors."""
    w, h, fx, fy, cx, cy = cam
    n = len(kps)
    sel = np.nonzero(rng.uniform(size=n) < keep)[0][:n_map]
    z = rng.uniform(2, 8, len(sel))
    X = np.stack([(kps["x"][sel] - cx) / fx * z, (kps["y"][sel] - cy) / fy * z, z], 1)
    nd = n_map - len(sel)
    zd = rng.uniform(2, 8, nd)
    Xd = np.stack([(rng.uniform(0, w, nd) - cx) / fx * zd, (rng.uniform(0, h, nd) - cy) / fy * zd, zd], 1)
    X = np.concatenate([X, Xd])
    sf = np.array([np.float32(scale) ** i for i in range(nlevels)], np.float64)
    lvl = np.concatenate([kps["octave"][sel], rng.integers(0, nlevels, nd)])
    dist = np.linalg.norm(X, axis=1)
    mp = np.zeros(n_map, MAP_POINT_DTYPE)
    mp["pos"] = X
    nrm = X / dist[:, None] + rng.normal(scale=0.01, size=X.shape)
    mp["normal"] = nrm / np.linalg.norm(nrm, axis=1, keepdims=True)
    mp["min_dist"] = dist / (sf[lvl] * 0.98)
    mp["max_dist"] = mp["min_dist"] * sf[-1] * 1.2
    mdesc = np.concatenate([synth.flip_bits(rng, desc[sel], max_flip),
                            rng.integers(0, 256, (nd, 32), dtype=np.uint8)])
    perm = rng.permutation(n_map)  # local-map order is arbitrary (Tracking.cc:3780-3821)
    return mp[perm], np.ascontiguousarray(mdesc[perm])


class FrontEnd:
    """B independent streams, one frame each per step."""

    def __init__(self, camera: str = "euroc", nfeatures: int = 1000, batch: int = 1, map_size: int = 2000,
                 nlevels: int = 8, scale: float = 1.2, fast_th: int = 20, ctx: Context | None = None, seed: int = 0):
        torch = _torch()
        self.cam = synth.CAMERAS[camera]
        self.B, self.M = batch, map_size
        w, h = self.cam[:2]
        self.ctx = ctx or Context(torch.cuda.current_device())
        self.ex = ORBextractor(nfeatures, scale, nlevels, 1, fast_th, width=w, height=h, max_batch=batch,
                               ctx=self.ctx)
        self.cap = self.ex.capacity
        self.info = FrameInfo.make(*self.cam, nlevels=nlevels, scale_factor=scale)
        dev = torch.device("cuda", self.ctx.device)
        self.stream = torch.cuda.Stream(device=dev)
        self.seed = seed
        B, cap, M = batch, self.cap, map_size
        u8, i32, f32 = torch.uint8, torch.int32, torch.float32
        self.imgs = torch.zeros((B, h, w), dtype=u8, device=dev)
        self.kps = torch.zeros((B, cap, KEYPOINT_DTYPE.itemsize), dtype=u8, device=dev)
        self.desc = torch.zeros((B, cap, 32), dtype=u8, device=dev)
        self.nkp = torch.zeros(B, dtype=i32, device=dev)
        self.mps = torch.zeros((B, M, MAP_POINT_DTYPE.itemsize), dtype=u8, device=dev)
        self.mp_desc = torch.zeros((B, M, 32), dtype=u8, device=dev)
        self.nmp = torch.full((B,), M, dtype=i32, device=dev)
        self.views = torch.zeros((B, M, MP_VIEW_DTYPE.itemsize), dtype=u8, device=dev)
        self.nview = torch.zeros(B, dtype=i32, device=dev)
        self.Tcw = torch.zeros((B, 16), dtype=f32, device=dev)
        self.kp2mp = torch.full((B, cap), -1, dtype=i32, device=dev)
        self.score = torch.full((B, cap), 999, dtype=i32, device=dev)
        self.nmatch = torch.zeros(B, dtype=i32, device=dev)

    # ------------------------------------------------------------ set-up
    def load_frames(self, frames: np.ndarray) -> None:
        torch = _torch()
        self.imgs.copy_(torch.from_numpy(np.ascontiguousarray(frames)))
        torch.cuda.synchronize()

    def build_maps(self, rot_deg: float = 0.05, trans: float = 0.002) -> None:
        """Extract once, then build every stream's local map and pose."""
        torch = _torch()
        self.extract()
        self.sync()
        kps = self.kps.cpu().numpy()
        desc = self.desc.cpu().numpy()
        nk = self.nkp.cpu().numpy()
        mps = np.zeros((self.B, self.M), MAP_POINT_DTYPE)
        mdesc = np.zeros((self.B, self.M, 32), np.uint8)
        T = np.zeros((self.B, 16), np.float32)
        for b in range(self.B):
            rng = np.random.default_rng(self.seed * 7919 + b)
            k = kps[b, :nk[b]].copy().view(KEYPOINT_DTYPE).reshape(-1)
            mps[b], mdesc[b] = build_local_map(k, desc[b, :nk[b]], self.cam, rng, self.M)
            T[b] = synth.look_pose(rng, trans, rot_deg).reshape(-1)
        self.mps.copy_(torch.from_numpy(mps.view(np.uint8).reshape(self.B, self.M, -1)))
        self.mp_desc.copy_(torch.from_numpy(mdesc))
        self.Tcw.copy_(torch.from_numpy(T))
        torch.cuda.synchronize()

    # ------------------------------------------------------------ stages
    @property
    def _s(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    def extract(self) -> None:
        self.ex.extract_batch_dev(self.imgs, self.kps, self.desc, self.nkp, stream=self.stream.cuda_stream)

    def frustum(self) -> None:
        check(lib().gf_frustum_dev(self.ctx.handle, ctypes.byref(self.info), self.B, ptr(self.Tcw), ptr(self.mps),
                                   ptr(self.nmp), self.M, ctypes.c_float(0.5), ptr(self.views), ptr(self.nview),
                                   self._s))

    def match_local_map(self, th: float = 1.0, nnratio: float = 0.8) -> None:
        self.kp2mp.fill_(-1)
        self.score.fill_(999)
        check(lib().gf_match_project_dev(self.ctx.handle, ctypes.byref(self.info), self.B, ptr(self.kps),
                                         ptr(self.desc), ptr(self.nkp), self.cap, ptr(self.views),
                                         ptr(self.mp_desc), ptr(self.nmp), self.M, ctypes.c_float(th),
                                         ctypes.c_float(nnratio), ptr(self.kp2mp), ptr(self.score),
                                         ptr(self.nmatch), self._s))

    def step(self) -> None:
        torch = _torch()
        with torch.cuda.stream(self.stream):
            self.extract()
            self.frustum()
            self.match_local_map()

    def sync(self) -> None:
        self.stream.synchronize()

    # ------------------------------------------------------------ profiling
    def prof_enable(self, on: bool = True) -> None:
        check(lib().gf_prof_enable(self.ctx.handle, int(on)))

    def prof_reset(self) -> None:
        check(lib().gf_prof_reset(self.ctx.handle))

    def prof_report(self) -> dict:
        out = {}
        i = 0
        name = ctypes.create_string_buffer(64)
        while True:
            ms, cnt = ctypes.c_double(), ctypes.c_int()
            rc = lib().gf_prof_report(self.ctx.handle, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt))
            if rc != 0:
                break
            out[name.value.decode()] = (ms.value, cnt.value)
            i += 1
        return out
