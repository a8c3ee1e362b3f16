"""Device-resident GF-ORB-SLAM front end for B independent streams on one GPU.

One `step()` runs the per-frame hot path of Tracking::GrabImageMonocular ->
Track() for every stream entirely on the device, through libgfslam's
device-family ABI, with no host round trip:

  ORB extraction (E1-E7)
  TrackWithMotionModel (Tracking.cc:1506-1570):
      Tcw = velocity * Tcw_last -> SearchByProjection(last frame) (M3)
      -> PoseOptimization (P1-P4) -> discard outliers
  TrackLocalMap / SearchReferencePointsInFrustum (Tracking.cc:3150-3340):
      updatePWLSVec (G1) -> FRAME_INFO_MATRIX over the matched points (G2-G4)
      -> mCurrentInfoMat (G5) -> isInFrustum over the local map (M7)
      -> MAP_INFO_MATRIX (G2-G4) -> runActiveMapMatching (G6/G7), or the
      plain SearchByProjection (M2) when gf=False
      -> PoseOptimization (P1-P4) -> discard outliers

The "last frame" state (keypoints, associations, pose, velocity) is fixed at
set-up so every step does the same work (a benchmark step, not a sequence).
PyTorch only provides device memory and the stream; all compute is in
libgfslam.so.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import synth
from ._lib import check, lib, ptr
from .matcher import MAP_POINT_DTYPE, MP_VIEW_DTYPE, FrameInfo
from .observability import ObsCamera, Rng
from .optimizer import inv_level_sigma2
from .orb import KEYPOINT_DTYPE, Context, ORBextractor


def _torch():
    import torch

    return torch


def build_local_map(kps: np.ndarray, desc: np.ndarray, cam, rng, n_map: int, scale: float = 1.2,
                    nlevels: int = 8, keep: float = 0.9, max_flip: int = 20, return_assoc: bool = False,
                    noise_px: float = 0.5):
    """Synthetic local map for one frame: most keypoints back-projected at a
    random depth (camera at the origin), descriptor = keypoint descriptor with
    a few flipped bits, plus distractor points with random descriptors. The
    back-projection is perturbed by N(0, noise_px) pixels so poses have a
    non-zero residual. With return_assoc, also the keypoint -> map index association (-1: none)."""
    w, h, fx, fy, cx, cy = cam
    n = len(kps)
    sel = np.nonzero(rng.uniform(size=n) < keep)[0][:n_map]
    z = rng.uniform(2, 8, len(sel))
    du = rng.normal(0, noise_px, (len(sel), 2)) if noise_px else np.zeros((len(sel), 2))
    X = np.stack([(kps["x"][sel] + du[:, 0] - cx) / fx * z, (kps["y"][sel] + du[:, 1] - cy) / fy * z, z], 1)
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
    if not return_assoc:
        return mp[perm], np.ascontiguousarray(mdesc[perm])
    inv = np.empty(n_map, np.int64)
    inv[perm] = np.arange(n_map)
    assoc = np.full(n, -1, np.int32)
    assoc[sel] = inv[np.arange(len(sel))]
    return mp[perm], np.ascontiguousarray(mdesc[perm]), assoc


class FrontEnd:
    """B independent streams, one frame each per step."""

    def __init__(self, camera: str = "euroc", nfeatures: int = 1000, batch: int = 1, map_size: int = 2000,
                 gf_budget: int = 100, last_matches: int = 60, gf: bool = True, nlevels: int = 8,
                 scale: float = 1.2, fast_th: int = 20, fps: float = 20.0, ctx: Context | None = None,
                 seed: int = 0):
        torch = _torch()
        self.cam = synth.CAMERAS[camera]
        self.B, self.M = batch, map_size
        self.gf, self.budget, self.last_matches, self.fps = gf, gf_budget, last_matches, fps
        w, h, fx, fy, cx, cy = self.cam
        self.ctx = ctx or Context(torch.cuda.current_device())
        self.ex = ORBextractor(nfeatures, scale, nlevels, 1, fast_th, width=w, height=h, max_batch=batch,
                               ctx=self.ctx)
        self.cap = self.ex.capacity
        self.info = FrameInfo.make(*self.cam, nlevels=nlevels, scale_factor=scale)
        self.obs_cam = ObsCamera.for_tracking(fx, fy, cx, cy, w, h)
        self.inv_sigma2 = inv_level_sigma2(nlevels, scale)
        sf = self.info.scale_factors()
        self.level_sigma2 = (sf * sf).astype(np.float32)  # Frame::mvLevelSigma2
        dev = torch.device("cuda", self.ctx.device)
        self.stream = torch.cuda.Stream(device=dev)
        self.seed = seed
        B, cap, M = batch, self.cap, map_size
        u8, i32, f32, f64 = torch.uint8, torch.int32, torch.float32, torch.float64
        z = lambda *s, dt=u8: torch.zeros(s, dtype=dt, device=dev)
        # current frame
        self.imgs = z(B, h, w)
        self.kps = z(B, cap, KEYPOINT_DTYPE.itemsize)
        self.desc = z(B, cap, 32)
        self.nkp = z(B, dt=i32)
        self.Tcw = z(B, 16, dt=f32)
        self.kp2mp = torch.full((B, cap), -1, dtype=i32, device=dev)
        self.score = torch.full((B, cap), 999, dtype=i32, device=dev)
        self.outl = z(B, cap)
        self.nmatch = z(B, dt=i32)
        self.ninl = z(B, dt=i32)
        self.iters = z(2, B, dt=i32)  # LM iterations of the two pose optimisations
        self.nedges = z(2, B, dt=i32)  # their edge counts (nInitialCorrespondences)
        self.num_to_match = z(B, dt=i32)
        self.scratch = z(B, cap, dt=i32)
        # last frame (fixed)
        self.last_kps = z(B, cap, KEYPOINT_DTYPE.itemsize)
        self.last_desc = z(B, cap, 32)
        self.last_nkp = z(B, dt=i32)
        self.last_kp2mp = torch.full((B, cap), -1, dtype=i32, device=dev)
        self.last_outl = z(B, cap)
        self.last_pos = z(B, cap, 3, dt=f32)
        self.Tcw_last = z(B, 16, dt=f32)
        self.velocity = z(B, 16, dt=f32)
        self.t_prev = z(B, dt=f64)
        self.t_cur = z(B, dt=f64)
        # local map
        self.mps = z(B, M, MAP_POINT_DTYPE.itemsize)
        self.mp_desc = z(B, M, 32)
        self.mp_pos = z(B, M, 3, dt=f32)
        self.nmp = torch.full((B,), M, dtype=i32, device=dev)
        self.views = z(B, M, MP_VIEW_DTYPE.itemsize)
        self.nview = z(B, dt=i32)
        # good-feature state: Xv of kinematic[0] / [1], mCurrentInfoMat, and the
        # map-resident MapPoint::H_meas / ObsMat / u_proj / updateAtFrameId
        self.Xv = z(B, 13, dt=f64)
        self.Xv_next = z(B, 13, dt=f64)
        self.base = z(B, 49, dt=f64)
        self.mp_H = z(B, M, 14, dt=f64)
        self.mp_info = z(B, M, 49, dt=f64)
        self.mp_uv = z(B, M, 2, dt=f32)
        self.mp_upd = torch.full((B, M), -1, dtype=i32, device=dev)
        self.mp_updated = z(B, M)
        self.frame_id = 1  # the current frame's stamp; stamps stay relative to it (see _step_body)
        self.graph = None
        self.rng = z(B, ctypes.sizeof(Rng), dt=u8)
        self.left = z(B, M, dt=i32)
        self.nleft = z(B, dt=i32)
        self.n_active = z(B, dt=i32)

    # ------------------------------------------------------------ set-up
    def load_frames(self, frames: np.ndarray) -> None:
        torch = _torch()
        self.imgs.copy_(torch.from_numpy(np.ascontiguousarray(frames)))
        torch.cuda.synchronize()

    def build_maps(self, rot_deg: float = 0.3, trans: float = 0.01) -> None:
        """Extract once, then build every stream's local map, the last frame
        (same view, `last_matches` associated keypoints, Tcw_last = I) and a
        small constant velocity."""
        torch = _torch()
        self.extract()
        self.sync()
        kps = self.kps.cpu().numpy()
        desc = self.desc.cpu().numpy()
        nk = self.nkp.cpu().numpy()
        B, M, cap = self.B, self.M, self.cap
        mps = np.zeros((B, M), MAP_POINT_DTYPE)
        mdesc = np.zeros((B, M, 32), np.uint8)
        last_kp2mp = np.full((B, cap), -1, np.int32)
        last_pos = np.zeros((B, cap, 3), np.float32)
        V = np.zeros((B, 16), np.float32)
        rngs = np.zeros((B, ctypes.sizeof(Rng)), np.uint8)
        for b in range(B):
            rng = np.random.default_rng(self.seed * 7919 + b)
            k = kps[b, :nk[b]].copy().view(KEYPOINT_DTYPE).reshape(-1)
            mps[b], mdesc[b], assoc = build_local_map(k, desc[b, :nk[b]], self.cam, rng, M, return_assoc=True)
            cand = np.nonzero(assoc >= 0)[0]
            keep = np.sort(rng.choice(cand, min(self.last_matches, len(cand)), replace=False))
            last_kp2mp[b, keep] = assoc[keep]
            last_pos[b, keep] = mps[b]["pos"][assoc[keep]]
            V[b] = synth.look_pose(rng, trans, rot_deg).reshape(-1)
            r = Rng.seeded(1 + self.seed * 1000 + b)
            rngs[b] = np.frombuffer(bytes(r), np.uint8)
        I = np.eye(4, dtype=np.float32).reshape(-1)
        self.last_kps.copy_(self.kps)
        self.last_desc.copy_(self.desc)
        self.last_nkp.copy_(self.nkp)
        self.last_kp2mp.copy_(torch.from_numpy(last_kp2mp))
        self.last_outl.zero_()
        self.last_pos.copy_(torch.from_numpy(last_pos))
        self.Tcw_last.copy_(torch.from_numpy(np.tile(I, (B, 1))))
        self.velocity.copy_(torch.from_numpy(V))
        self.t_prev.fill_(0.0)
        self.t_cur.fill_(1.0 / self.fps)
        self.mps.copy_(torch.from_numpy(mps.view(np.uint8).reshape(B, M, -1)))
        self.mp_desc.copy_(torch.from_numpy(mdesc))
        self.mp_pos.copy_(torch.from_numpy(np.ascontiguousarray(mps["pos"])))
        self.rng0 = torch.from_numpy(rngs).to(self.rng.device)
        self.rng.copy_(self.rng0)
        torch.cuda.synchronize()

    # ------------------------------------------------------------ stages
    @property
    def _s(self):
        return ctypes.c_void_p(self.stream.cuda_stream)

    @property
    def _h(self):
        return self.ctx.handle

    def extract(self) -> None:
        self.ex.extract_batch_dev(self.imgs, self.kps, self.desc, self.nkp, stream=self.stream.cuda_stream)

    def predict_pose(self) -> None:
        check(lib().gf_motion_predict_dev(self._h, self.B, ptr(self.velocity), ptr(self.Tcw_last), ptr(self.Tcw),
                                          self._s))

    def reset_matches(self) -> None:
        self.kp2mp.fill_(-1)
        self.score.fill_(999)
        self.outl.zero_()

    def match_last_frame(self, th: float = 15.0) -> None:
        """ORBmatcher(0.9, true).SearchByProjection(mCurrentFrame, mLastFrame, 15)."""
        check(lib().gf_match_lastframe_dev(self._h, ctypes.byref(self.info), self.B, ptr(self.kps), ptr(self.desc),
                                           ptr(self.nkp), self.cap, ptr(self.Tcw), ptr(self.last_kps),
                                           ptr(self.last_desc), ptr(self.last_kp2mp), ptr(self.last_outl),
                                           ptr(self.last_pos), ptr(self.last_nkp), self.cap, ctypes.c_float(th), 1,
                                           ptr(self.kp2mp), ptr(self.score), ptr(self.nmatch), ptr(self.scratch),
                                           self._s))

    def pose_optimization(self, which: int = 0) -> None:
        fi = self.info
        check(lib().gf_pose_opt_frames_dev(self._h, self.B, ptr(self.Tcw), ptr(self.kps), ptr(self.nkp), self.cap,
                                           ptr(self.kp2mp), ptr(self.mps), self.M, ptr(self.inv_sigma2),
                                           len(self.inv_sigma2), ctypes.c_float(fi.fx), ctypes.c_float(fi.fy),
                                           ctypes.c_float(fi.cx), ctypes.c_float(fi.cy), ptr(self.outl),
                                           ptr(self.ninl), ptr(self.iters[which]), ptr(self.nedges[which]),
                                           self._s))

    def discard_outliers(self) -> None:
        check(lib().gf_discard_outliers_dev(self._h, self.B, ptr(self.kp2mp), ptr(self.outl), ptr(self.nkp),
                                            self.cap, self.budget, ptr(self.nmatch), ptr(self.num_to_match),
                                            self._s))

    def frame_info(self) -> None:
        """SearchReferencePointsInFrustum head (Tracking.cc:3160-3213): G1 at the
        motion-model pose, FRAME_INFO_MATRIX over the matched points and
        mCurrentInfoMat from the ones stamped for this frame."""
        check(lib().gf_obs_update_dev(self._h, self.B, ptr(self.t_prev), ptr(self.Tcw_last), ptr(self.t_cur),
                                      ptr(self.Tcw), ptr(self.Xv), None, self._s))
        check(lib().gf_obs_frame_info_dev(self._h, ctypes.byref(self.obs_cam), self.B, ptr(self.Xv), ptr(self.kps),
                                          ptr(self.nkp), self.cap, ptr(self.kp2mp), ptr(self.outl), ptr(self.mp_pos),
                                          ptr(self.nmp), self.M, ptr(self.level_sigma2), len(self.level_sigma2),
                                          ptr(self.mp_H), ptr(self.mp_info), ptr(self.mp_uv), self._s))
        check(lib().gf_obs_accumulate_matched_dev(self._h, self.B, ptr(self.kp2mp), ptr(self.nkp), self.cap,
                                                  ptr(self.mp_info), ptr(self.mp_upd), ptr(self.nmp), self.M,
                                                  self.frame_id, ctypes.c_double(1e-5), ptr(self.base), self._s))

    def frustum(self) -> None:
        check(lib().gf_frustum_dev(self._h, ctypes.byref(self.info), self.B, ptr(self.Tcw), ptr(self.mps),
                                   ptr(self.nmp), self.M, ctypes.c_float(0.5), ptr(self.views), ptr(self.nview),
                                   self._s))
        check(lib().gf_views_exclude_matched_dev(self._h, self.B, ptr(self.kp2mp), ptr(self.nkp), self.cap,
                                                 ptr(self.views), ptr(self.nmp), self.M, self._s))

    def map_info(self) -> None:
        """MAP_INFO_MATRIX for the visible points not yet stamped this frame."""
        check(lib().gf_obs_map_info_dev(self._h, ctypes.byref(self.obs_cam), self.B, ptr(self.Xv), ptr(self.mp_pos),
                                        ptr(self.nmp), self.M, 0, ptr(self.views), ptr(self.mp_upd), self.frame_id,
                                        ptr(self.mp_H), ptr(self.mp_info), ptr(self.mp_uv), ptr(self.mp_updated),
                                        self._s))

    def predict_next(self) -> None:
        """After TrackLocalMap: updatePWLSVec at the final pose, predict 2
        segments (Tracking.cc:795-800) and build the map information for the
        next frame at kinematic[1] with the visibility check
        (RunMapPointsSelection, Tracking.cc:1717-1772)."""
        check(lib().gf_obs_update_dev(self._h, self.B, ptr(self.t_prev), ptr(self.Tcw_last), ptr(self.t_cur),
                                      ptr(self.Tcw), ptr(self.Xv), ptr(self.Xv_next), self._s))
        check(lib().gf_obs_map_info_dev(self._h, ctypes.byref(self.obs_cam), self.B, ptr(self.Xv_next),
                                        ptr(self.mp_pos), ptr(self.nmp), self.M, 1, None, ptr(self.mp_upd),
                                        self.frame_id + 1, ptr(self.mp_H), ptr(self.mp_info), ptr(self.mp_uv), None,
                                        self._s))

    def active_match(self, th: float = 1.0, nnratio: float = 0.8) -> None:
        check(lib().gf_obs_active_match_dev(self._h, ctypes.byref(self.info), self.B, ptr(self.kps), ptr(self.desc),
                                            ptr(self.nkp), self.cap, ptr(self.views), ptr(self.mp_desc),
                                            ptr(self.mp_updated), ptr(self.mp_info), ptr(self.mp_H), ptr(self.nmp),
                                            self.M, ptr(self.base), ptr(self.level_sigma2), ptr(self.num_to_match),
                                            ctypes.c_float(th), ctypes.c_float(nnratio), ptr(self.rng),
                                            ptr(self.kp2mp), ptr(self.score), ptr(self.left), ptr(self.nleft),
                                            ptr(self.n_active), self._s))

    def match_local_map(self, th: float = 1.0, nnratio: float = 0.8) -> None:
        check(lib().gf_match_project_dev(self._h, ctypes.byref(self.info), self.B, ptr(self.kps), ptr(self.desc),
                                         ptr(self.nkp), self.cap, ptr(self.views), ptr(self.mp_desc), ptr(self.nmp),
                                         self.M, ctypes.c_float(th), ctypes.c_float(nnratio), ptr(self.kp2mp),
                                         ptr(self.score), ptr(self.n_active), self._s))

    def _step_body(self) -> None:
        self.extract()
        # TrackWithMotionModel
        self.predict_pose()
        self.reset_matches()
        self.match_last_frame()
        self.pose_optimization(0)
        self.discard_outliers()
        # TrackLocalMap -> SearchReferencePointsInFrustum
        if self.gf:
            self.frame_info()
        self.frustum()
        if self.gf:
            self.map_info()
            self.active_match()
        else:
            self.match_local_map()
        self.pose_optimization(1)
        self.discard_outliers()
        if self.gf:
            self.predict_next()
        # MapPoint::updateAtFrameId stamps are kept relative to the current
        # frame: this frame is always frame_id (1) and the next frame_id + 1, so
        # after a step every stamp moves down by one. The kernels only compare
        # stamps for equality with the current / next id, so this is the
        # reference's absolute mnId bookkeeping, and a step has no per-frame
        # host arguments (it can be captured once as a HIP graph and replayed).
        self.mp_upd.sub_(1)

    def step(self) -> None:
        torch = _torch()
        if self.graph is not None:
            self.graph.replay()
            return
        with torch.cuda.stream(self.stream):
            self._step_body()

    def capture_graph(self) -> None:
        """Capture one step as a HIP graph (after at least one eager step, so
        every workspace is allocated); step() replays it from then on.
        Measured on ROCm 7.2 (scripts/overlap_exp.py): replaying per-group
        graphs is slower than eager launches on two streams (61.6k vs 73.4k
        frames/s at 512 streams), because the replays do not overlap across
        streams; the bench therefore launches eagerly."""
        torch = _torch()
        self.sync()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=self.stream):
            self._step_body()
        self.graph = g  # capturing records the step without running it

    def reset_state(self) -> None:
        """Back to the state right after build_maps (RNG, map stamps, frame id)."""
        self.rng.copy_(self.rng0)
        self.mp_upd.fill_(-1)
        self.frame_id = 1

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
