"""Synthetic sequences for the tracking front end.

No dataset is reachable from the build or the GPU box, so sequences are
rendered: a room of textured planes (walls, floor, ceiling and two
free-standing panels) seen by a pinhole camera that moves on a closed
trajectory of `period` frames (dt = 1/fps), so a stream can be tracked for
any number of steps. Frames are rendered with torch (plumbing: on the GPU
for the bench, on the CPU for host tests); the same ray-plane geometry in
float64 back-projects keyframe keypoints into the map points of the scene's
local map, as a keyframe-built map of the reference would hold them
(MapPoint::UpdateNormalAndDepth, MapPoint.cc:285-326, for the normal and the
scale-invariance distances).

Each stream b tracks scene b % n_scenes from phase (b // n_scenes) * stride
of the loop; its first frame initialises the tracker at the ground-truth pose
(gf_frontend_bootstrap), with the constant-velocity motion of the previous
frame.
"""
from __future__ import annotations

import math

import numpy as np

from . import synth


def _rot(ax: str, a: float) -> np.ndarray:
    c, s = math.cos(a), math.sin(a)
    if ax == "x":
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if ax == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


class Scene:
    """Textured planes: origin o, unit axes u, v, extents (su, sv) in metres."""

    def __init__(self, seed: int, tex_size: int = 1024):
        rng = np.random.default_rng(seed)
        j = lambda s: float(rng.uniform(-s, s))
        planes = [  # (o, u, v, su, sv)
            ((-5.0, -3.5, 6.0 + j(0.5)), (1, 0, 0), (0, 1, 0), 10.0, 7.0),   # back wall
            ((-5.0, 1.6 + j(0.2), 0.3), (1, 0, 0), (0, 0, 1), 10.0, 7.0),    # floor
            ((-5.0, -2.2 + j(0.2), 0.3), (1, 0, 0), (0, 0, 1), 10.0, 7.0),   # ceiling
            ((-3.5 + j(0.3), -3.5, 0.3), (0, 0, 1), (0, 1, 0), 7.0, 7.0),    # left wall
            ((3.5 + j(0.3), -3.5, 0.3), (0, 0, 1), (0, 1, 0), 7.0, 7.0),     # right wall
            ((-1.6 + j(0.3), -0.7 + j(0.2), 3.2 + j(0.3)), (1, 0, 0), (0, 1, 0), 1.4, 1.3),  # panel
            ((0.6 + j(0.3), -0.2 + j(0.2), 4.3 + j(0.3)), (1, 0, 0), (0, 1, 0), 1.6, 1.4),   # panel
        ]
        self.o = np.array([p[0] for p in planes], np.float64)
        self.u = np.array([p[1] for p in planes], np.float64)
        self.v = np.array([p[2] for p in planes], np.float64)
        self.su = np.array([p[3] for p in planes], np.float64)
        self.sv = np.array([p[4] for p in planes], np.float64)
        self.n = np.cross(self.u, self.v)
        self.tex_size = tex_size
        nshape = int(400 * tex_size * tex_size / (752 * 480))
        self.textures = np.stack([synth.synth_frame(tex_size, tex_size, seed * 100 + k, n_shapes=nshape)
                                  for k in range(len(planes))])

    # --------------------------------------------------------- transport
    def pack(self) -> np.ndarray:
        """One byte blob (plane geometry f64 + textures u8), for the start-up broadcast."""
        geo = np.concatenate([self.o.ravel(), self.u.ravel(), self.v.ravel(), self.su, self.sv])
        hdr = np.array([len(self.o), self.tex_size], np.int64)
        return np.concatenate([hdr.view(np.uint8), geo.view(np.uint8), self.textures.reshape(-1)])

    @classmethod
    def unpack(cls, blob: np.ndarray) -> "Scene":
        P, T = (int(x) for x in blob[:16].view(np.int64))
        geo = blob[16:16 + 8 * 11 * P].view(np.float64)
        sc = cls.__new__(cls)
        sc.o, sc.u, sc.v = geo[:3 * P].reshape(P, 3), geo[3 * P:6 * P].reshape(P, 3), geo[6 * P:9 * P].reshape(P, 3)
        sc.su, sc.sv = geo[9 * P:10 * P].copy(), geo[10 * P:11 * P].copy()
        sc.n = np.cross(sc.u, sc.v)
        sc.tex_size = T
        sc.textures = blob[16 + 8 * 11 * P:].reshape(P, T, T).copy()
        return sc

    # --------------------------------------------------------- geometry
    def intersect(self, C: np.ndarray, d: np.ndarray):
        """Nearest plane hit of rays C + lam d (d: [N, 3]), float64: returns
        (lam [N], plane [N], a [N], b [N]); plane -1 = no hit."""
        N = len(d)
        best = np.full(N, np.inf)
        pid = np.full(N, -1, np.int64)
        A = np.zeros(N)
        Bc = np.zeros(N)
        for k in range(len(self.o)):
            den = d @ self.n[k]
            with np.errstate(divide="ignore", invalid="ignore"):
                lam = ((self.o[k] - C) @ self.n[k]) / den
            X = C + lam[:, None] * d
            a = (X - self.o[k]) @ self.u[k]
            b = (X - self.o[k]) @ self.v[k]
            ok = (lam > 1e-6) & (a >= 0) & (a <= self.su[k]) & (b >= 0) & (b <= self.sv[k]) & (lam < best)
            best[ok], pid[ok], A[ok], Bc[ok] = lam[ok], k, a[ok], b[ok]
        return best, pid, A, Bc

    def backproject(self, Tcw: np.ndarray, x: np.ndarray, y: np.ndarray, cam, dist=None) -> tuple:
        """World points of pixels (x, y) seen from Tcw; valid mask. dist: the
        pixels are in a distorted image (radial-tangential k1 k2 p1 p2 [k3])."""
        _, _, fx, fy, cx, cy = cam
        T = np.asarray(Tcw, np.float64)
        R, t = T[:3, :3], T[:3, 3]
        C = -R.T @ t
        xn, yn = (x - cx) / fx, (y - cy) / fy
        if dist is not None:
            xn, yn = synth.undistort_normalized(xn, yn, dist)
        dc = np.stack([xn, yn, np.ones_like(x, dtype=np.float64)], 1)
        dw = dc @ R  # R^T d
        lam, pid, _, _ = self.intersect(C, dw)
        X = C + lam[:, None] * dw
        return X, pid >= 0

    def render(self, Tcws, cam, device="cpu", dist=None):
        """u8 frames [N][H][W] for N poses (torch on `device`); dist: a
        distorted image (radial-tangential k1 k2 p1 p2 [k3])."""
        import torch
        import torch.nn.functional as Fn

        w, h, fx, fy, cx, cy = cam
        dev = torch.device(device)
        tex = torch.from_numpy(self.textures).to(dev).float()[:, None]  # [P,1,T,T]
        if dist is None:
            ys, xs = torch.meshgrid(torch.arange(h, device=dev, dtype=torch.float32),
                                    torch.arange(w, device=dev, dtype=torch.float32), indexing="ij")
            dc = torch.stack([(xs - cx) / fx, (ys - cy) / fy, torch.ones_like(xs)], -1).reshape(-1, 3)
        else:  # each pixel's ray through the ideal (undistorted) normalised point
            ys, xs = np.meshgrid(np.arange(h, dtype=np.float64), np.arange(w, dtype=np.float64), indexing="ij")
            xn, yn = synth.undistort_normalized((xs - cx) / fx, (ys - cy) / fy, dist)
            dc = torch.from_numpy(np.stack([xn, yn, np.ones_like(xn)], -1).reshape(-1, 3).astype(np.float32)).to(dev)
        out = []
        o = torch.from_numpy(self.o).float().to(dev)
        u = torch.from_numpy(self.u).float().to(dev)
        v = torch.from_numpy(self.v).float().to(dev)
        n = torch.from_numpy(self.n).float().to(dev)
        su = torch.from_numpy(self.su).float().to(dev)
        sv = torch.from_numpy(self.sv).float().to(dev)
        for T in Tcws:
            T = np.asarray(T, np.float64)
            R = torch.from_numpy(T[:3, :3]).float().to(dev)
            C = torch.from_numpy(-T[:3, :3].T @ T[:3, 3]).float().to(dev)
            dw = dc @ R
            best = torch.full((dw.shape[0],), float("inf"), device=dev)
            val = torch.zeros(dw.shape[0], device=dev)
            for k in range(len(self.o)):
                den = dw @ n[k]
                lam = ((o[k] - C) @ n[k]) / den
                X = C + lam[:, None] * dw
                a = (X - o[k]) @ u[k]
                b = (X - o[k]) @ v[k]
                ok = (lam > 1e-6) & (a >= 0) & (a <= su[k]) & (b >= 0) & (b <= sv[k]) & (lam < best)
                g = torch.stack([a / su[k] * 2 - 1, b / sv[k] * 2 - 1], -1).reshape(1, 1, -1, 2)
                s = Fn.grid_sample(tex[k:k + 1], g, mode="bilinear", align_corners=True).reshape(-1)
                best = torch.where(ok, lam, best)
                val = torch.where(ok, s, val)
            out.append(torch.clamp(torch.round(val), 0, 255).to(torch.uint8).reshape(h, w))
        return torch.stack(out)


# ------------------------------------------------------------- trajectory
def trajectory_pose(phase: float, period: int, seed: int = 0) -> np.ndarray:
    """Tcw (float32 4x4) at a phase of the closed loop (EuRoC-like speed:
    about 1 m/s and 15 deg/s at dt = 0.05, period 32)."""
    rng = np.random.default_rng(seed)
    a0, a1, a2 = rng.uniform(0, 2 * math.pi, 3)
    th = 2 * math.pi * phase / period
    C = np.array([0.25 * math.sin(th + a0), 0.08 * math.sin(2 * th + a1), 0.15 * (1 - math.cos(th + a2))])
    Rwc = _rot("y", 0.06 * math.sin(th + 0.5 + a1)) @ _rot("x", 0.03 * math.sin(2 * th + a2)) @ \
        _rot("z", 0.01 * math.sin(th + a0))
    T = np.eye(4)
    T[:3, :3] = Rwc.T
    T[:3, 3] = -Rwc.T @ C
    return T.astype(np.float32)


def velocity(T_prev: np.ndarray, T_cur: np.ndarray) -> np.ndarray:
    """mVelocity = Tcw_cur * Twc_prev (Tracking.cc:735), float32."""
    return (T_cur.astype(np.float64) @ np.linalg.inv(T_prev.astype(np.float64))).astype(np.float32)


# ------------------------------------------------------------- local map
def build_map(scene: Scene, cam, extract, period: int, traj_seed: int, n_map: int, seed: int,
              n_kf: int = 8, nlevels: int = 8, scale: float = 1.2, device="cpu", stale_desc: float = 0.0,
              dist=None):
    """Map points from n_kf keyframes along the loop: every keypoint of a
    keyframe back-projected onto the scene (duplicates within 2 cm merged,
    first keyframe wins), the keyframe descriptor, normal and the
    scale-invariance distances of UpdateNormalAndDepth. Returns
    (MAP_POINT_DTYPE array, descriptors), at most n_map points in a seeded
    arbitrary order (the reference's std::map<KeyFrame*> pointer order).
    `extract(img) -> (keypoints, descriptors)`.

    stale_desc: fraction of the points whose descriptor no longer describes
    them: a seeded random 256-bit descriptor (Bernoulli 0.5 bits, SURVEY.md
    §8d's map-descriptor model). These points project into view and enter
    every visibility and information computation but can practically never
    be matched (Hamming distance to any keypoint ~128 +- 8 > TH_HIGH = 100),
    as local-map points triangulated from distant keyframes are in a real
    sequence. It sets how many matches a frame
    carries to the next one, hence the SearchReferencePointsInFrustum branch:
    config 2's recipe (about 60 last-frame matches against GF
    budget 100, so runActiveMapMatching runs every frame) is stale_desc = 0.94
    (bench.py --stale-desc)."""
    from .matcher import MAP_POINT_DTYPE

    sf = [np.float32(1.0)]
    for _ in range(1, nlevels):
        sf.append(np.float32(sf[-1] * np.float32(scale)))
    sf = np.array(sf, np.float32)
    poses = [trajectory_pose(k * period / n_kf, period, traj_seed) for k in range(n_kf)]
    imgs = scene.render(poses, cam, device, dist=dist).cpu().numpy()
    Xs, Ds, Ns, dmin, dmax = [], [], [], [], []
    for T, img in zip(poses, imgs):
        k, d = extract(img)
        X, ok = scene.backproject(T, k["x"].astype(np.float64), k["y"].astype(np.float64), cam, dist=dist)
        C = -T[:3, :3].astype(np.float64).T @ T[:3, 3].astype(np.float64)
        X, d, oc = X[ok], d[ok], k["octave"][ok]
        PC = (X - C).astype(np.float32)
        dpc = np.sqrt((PC.astype(np.float64) ** 2).sum(1)).astype(np.float32)
        Xs.append(X)
        Ds.append(d)
        Ns.append(PC / dpc[:, None])
        lvl = sf[oc]
        dmin.append((np.float32(1.0) / np.float32(scale)) * dpc / lvl)
        dmax.append(np.float32(scale) * dpc * sf[nlevels - 1 - oc])
    X = np.concatenate(Xs)
    D = np.concatenate(Ds)
    keys = np.floor(X / 0.02).astype(np.int64)
    _, first = np.unique(keys, axis=0, return_index=True)
    keep = np.sort(first)
    rng = np.random.default_rng(seed)
    keep = rng.permutation(keep)[:n_map]
    mp = np.zeros(len(keep), MAP_POINT_DTYPE)
    mp["pos"] = X[keep]
    mp["normal"] = np.concatenate(Ns)[keep]
    mp["min_dist"] = np.concatenate(dmin)[keep]
    mp["max_dist"] = np.concatenate(dmax)[keep]
    D = np.ascontiguousarray(D[keep])
    if stale_desc > 0:
        srng = np.random.default_rng(seed + 0x5747)
        sel = srng.permutation(len(keep))[:int(round(stale_desc * len(keep)))]
        D[sel] = srng.integers(0, 256, (len(sel), 32), dtype=np.uint8)
    return mp, D


def keyframe_pose(k: int, n_kf: int, period: int, traj_seed: int, sweep: float) -> np.ndarray:
    """Keyframe k of a mapping sweep: the loop's position at phase k period /
    n_kf, turned about the vertical axis by a yaw spread evenly over
    [-sweep, +sweep] rad (the mapping pass looked around the room; the
    tracked loop looks ahead)."""
    T = trajectory_pose(k * period / n_kf, period, traj_seed).astype(np.float64)
    yaw = -sweep + 2 * sweep * k / max(n_kf - 1, 1)
    Rwc = T[:3, :3].T @ _rot("y", yaw)
    C = -T[:3, :3].T @ T[:3, 3]
    out = np.eye(4)
    out[:3, :3] = Rwc.T
    out[:3, 3] = -Rwc.T @ C
    return out.astype(np.float32)


def build_global_map(scene: Scene, cam, extract, period: int, traj_seed: int, g_cap: int, seed: int, n_kf: int = 24,
                     nlevels: int = 8, scale: float = 1.2, device="cpu", stale_desc: float = 0.0,
                     min_shared: int = 15, sweep: float = 2.4) -> dict:
    """A keyframe map for Tracking::UpdateReference: n_kf keyframes of a
    mapping sweep (keyframe_pose), every keypoint back-projected onto the
    scene; a
    keypoint whose 3-D point falls within 2 cm of an existing map point becomes
    an observation of it (one slot per keyframe and point), else a new point
    (its keyframe's descriptor, normal and UpdateNormalAndDepth distances, as
    build_map). At most g_cap points are kept (a seeded subset, in a seeded
    order: the map's point indices); slots of dropped points are NULL. The
    keyframes' keypoints and descriptors (kf_kps / kf_desc, slot order) feed
    the relocalisation keyframe database (pipeline.KeyframeDB).
    Keyframes are in creation order (= ascending KeyFrame*); each keyframe's
    covisible keyframes sharing >= min_shared points, by weight descending
    (ties: later keyframe first), are mvpOrderedConnectedKeyFrames
    (KeyFrame::UpdateConnections, KeyFrame.cc). stale_desc as build_map.
    Returns dict(mp, desc, graph=localmap.CovisGraph arrays, kf_Tcw)."""
    from .matcher import MAP_POINT_DTYPE

    sf = [np.float32(1.0)]
    for _ in range(1, nlevels):
        sf.append(np.float32(sf[-1] * np.float32(scale)))
    sf = np.array(sf, np.float32)
    poses = [keyframe_pose(k, n_kf, period, traj_seed, sweep) for k in range(n_kf)]
    imgs = scene.render(poses, cam, device).cpu().numpy()
    key_to_pt = {}
    X_l, D_l, N_l, dmin_l, dmax_l = [], [], [], [], []
    slots = []  # per keyframe: point id per keypoint slot (-1 = NULL)
    kf_kps, kf_desc = [], []
    for T, img in zip(poses, imgs):
        k, d = extract(img)
        kf_kps.append(k)
        kf_desc.append(d)
        X, ok = scene.backproject(T, k["x"].astype(np.float64), k["y"].astype(np.float64), cam)
        C = -T[:3, :3].astype(np.float64).T @ T[:3, 3].astype(np.float64)
        sl = np.full(len(k), -1, np.int64)
        seen = set()
        for i in np.nonzero(ok)[0]:
            key = tuple(np.floor(X[i] / 0.02).astype(np.int64))
            pid = key_to_pt.get(key)
            if pid is None:
                pid = len(X_l)
                key_to_pt[key] = pid
                PC = (X[i] - C).astype(np.float32)
                dist = np.float32(np.sqrt((PC.astype(np.float64) ** 2).sum()))
                X_l.append(X[i])
                D_l.append(d[i])
                N_l.append(PC / dist)
                oc = int(k["octave"][i])
                dmin_l.append((np.float32(1.0) / np.float32(scale)) * dist / sf[oc])
                dmax_l.append(np.float32(scale) * dist * sf[nlevels - 1 - oc])
            if pid in seen:
                continue  # one slot per keyframe and point
            seen.add(pid)
            sl[i] = pid
        slots.append(sl)
    npt = len(X_l)
    rng = np.random.default_rng(seed)
    keep = rng.permutation(npt)[:g_cap]  # kept points, in their new index order
    newid = np.full(npt, -1, np.int64)
    newid[keep] = np.arange(len(keep))
    G = len(keep)
    mp = np.zeros(G, MAP_POINT_DTYPE)
    mp["pos"] = np.array(X_l)[keep]
    mp["normal"] = np.array(N_l)[keep]
    mp["min_dist"] = np.array(dmin_l, np.float32)[keep]
    mp["max_dist"] = np.array(dmax_l, np.float32)[keep]
    desc = np.ascontiguousarray(np.array(D_l, np.uint8)[keep])
    if stale_desc > 0:
        srng = np.random.default_rng(seed + 0x5747)
        sel = srng.permutation(G)[:int(round(stale_desc * G))]
        desc[sel] = srng.integers(0, 256, (len(sel), 32), dtype=np.uint8)
    kf_mp = [np.where(sl >= 0, newid[np.maximum(sl, 0)], -1).astype(np.int32) for sl in slots]
    kf_mp_off = np.zeros(n_kf + 1, np.int32)
    kf_mp_off[1:] = np.cumsum([len(x) for x in kf_mp])
    obs = [[] for _ in range(G)]
    for kf, x in enumerate(kf_mp):
        for m in x[x >= 0]:
            obs[m].append(kf)
    mp_obs_off = np.zeros(G + 1, np.int32)
    mp_obs_off[1:] = np.cumsum([len(o) for o in obs])
    shared = np.zeros((n_kf, n_kf), np.int64)
    for o in obs:
        for a in o:
            for b in o:
                if a != b:
                    shared[a, b] += 1
    cov = []
    for a in range(n_kf):
        nb = [b for b in range(n_kf) if b != a and shared[a, b] >= min_shared]
        cov.append(sorted(nb, key=lambda b: (-shared[a, b], -b)))
    kf_cov_off = np.zeros(n_kf + 1, np.int32)
    kf_cov_off[1:] = np.cumsum([len(c) for c in cov])
    graph = dict(kf_bad=np.zeros(n_kf, np.uint8), kf_mp_off=kf_mp_off, kf_mp=np.concatenate(kf_mp),
                 kf_cov_off=kf_cov_off, kf_cov=np.array([b for c in cov for b in c], np.int32),
                 mp_bad=np.zeros(G, np.uint8), mp_obs_off=mp_obs_off,
                 mp_obs=np.array([k for o in obs for k in o], np.int32))
    return dict(mp=mp, desc=desc, graph=graph, kf_Tcw=np.stack(poses), kf_kps=kf_kps, kf_desc=kf_desc)


class Workload:
    """B streams over n_scenes rendered loops (see module docstring)."""

    def __init__(self, camera: str, batch: int, n_scenes: int = 8, period: int = 32, seed: int = 0,
                 phase_stride: int = 5, tex_size: int = 1024, scenes: list | None = None, phase_offset: int = 0,
                 stale_desc: float = 0.0, dist=None):
        self.cam = synth.CAMERAS[camera]
        self.dist = dist  # radial-tangential coefficients of distorted renders (None: pinhole)
        self.stale_desc = stale_desc
        self.B, self.S, self.period, self.seed = batch, min(n_scenes, batch), period, seed
        self.scenes = scenes if scenes is not None else [Scene(seed * 1000 + s, tex_size) for s in range(self.S)]
        self.scene_of = np.arange(batch) % self.S
        self.phase = ((np.arange(batch) // self.S) * phase_stride + seed + phase_offset) % period
        self.traj_seed = [seed * 1000 + s for s in range(self.S)]

    def render_all(self, device="cpu"):
        """[S][period][H][W] u8 frames (torch, on `device`)."""
        import torch

        frames = []
        for s, sc in enumerate(self.scenes):
            poses = [trajectory_pose(k, self.period, self.traj_seed[s]) for k in range(self.period)]
            frames.append(sc.render(poses, self.cam, device, dist=self.dist))
        return torch.stack(frames)

    def gt_pose(self, stream: int, step: int) -> np.ndarray:
        """Ground-truth Tcw of a stream's frame at a step (step 0 = bootstrap)."""
        s = self.scene_of[stream]
        return trajectory_pose((self.phase[stream] + step) % self.period, self.period, self.traj_seed[s])

    def boot_state(self):
        """Tcw [B][16] of the bootstrap frame and the constant-velocity V [B][16]."""
        T = np.stack([self.gt_pose(b, 0).reshape(16) for b in range(self.B)])
        V = np.stack([velocity(self.gt_pose(b, -1), self.gt_pose(b, 0)).reshape(16) for b in range(self.B)])
        return np.ascontiguousarray(T, np.float32), np.ascontiguousarray(V, np.float32)

    def build_global_maps(self, extract, g_cap: int, n_kf: int = 24, device="cpu", sweep: float = 2.4):
        """Per scene: build_global_map (keyframes, covisibility, points) for
        local maps assembled per frame by UpdateReference."""
        return [build_global_map(sc, self.cam, extract, self.period, self.traj_seed[s], g_cap, self.seed * 7919 + s,
                                 n_kf=n_kf, device=device, stale_desc=self.stale_desc, sweep=sweep)
                for s, sc in enumerate(self.scenes)]

    def build_maps(self, extract, n_map: int, device="cpu"):
        return [build_map(sc, self.cam, extract, self.period, self.traj_seed[s], n_map, self.seed * 7919 + s,
                          device=device, stale_desc=self.stale_desc, dist=self.dist)
                for s, sc in enumerate(self.scenes)]
