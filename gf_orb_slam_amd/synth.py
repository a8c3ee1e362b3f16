"""Seeded synthetic inputs. No datasets are reachable from the
build or the GPU box, so every benchmark and parity case runs on these.

Frames: 2-octave value noise + ~400 uniform rectangles/discs, Gaussian
sigma 0.8 pre-smoothing, uniform noise +-3, clipped to u8. Seeds follow
0x6F52420 + stream*1000 + frame.
"""
from __future__ import annotations

import numpy as np

CAMERAS = {
    # name: (width, height, fx, fy, cx, cy)
    "euroc": (752, 480, 457.3, 457.3, 367.215, 248.375),
    "tum": (640, 480, 525.0, 525.0, 319.5, 239.5),
}
# radial-tangential coefficients k1 k2 p1 p2 of real cameras (the public
# EuRoC MAV cam0 and TUM fr2 calibrations), for distorted renders
DISTORTION = {
    "euroc": (-0.28340811, 0.07395907, 0.00019359, 1.76187114e-05),
    "tum": (0.231222, -0.784899, -0.003257, -0.000105, 0.917205),
}


def undistort_normalized(xd, yd, dist, iters: int = 20):
    """Ideal normalised coordinates of distorted normalised ones (fixed-point
    inversion of the radial-tangential model, float64; for rendering and map
    building only — the tracked keypoints go through cv::undistortPoints'
    restatement in the library)."""
    k1, k2, p1, p2, k3 = (list(dist) + [0.0] * 5)[:5]
    x, y = xd.copy(), yd.copy()
    for _ in range(iters):
        r2 = x * x + y * y
        rad = 1 + ((k3 * r2 + k2) * r2 + k1) * r2
        dx = 2 * p1 * x * y + p2 * (r2 + 2 * x * x)
        dy = p1 * (r2 + 2 * y * y) + 2 * p2 * x * y
        x = (xd - dx) / rad
        y = (yd - dy) / rad
    return x, y


def frame_seed(stream: int, frame: int) -> int:
    return 0x6F52420 + stream * 1000 + frame


def _value_noise(rng, h, w, cell):
    gh, gw = h // cell + 2, w // cell + 2
    g = rng.uniform(0, 1, (gh, gw)).astype(np.float32)
    ys = np.arange(h, dtype=np.float32) / cell
    xs = np.arange(w, dtype=np.float32) / cell
    y0, x0 = ys.astype(int), xs.astype(int)
    fy, fx = (ys - y0)[:, None], (xs - x0)[None, :]
    a = g[y0][:, x0]
    b = g[y0][:, x0 + 1]
    c = g[y0 + 1][:, x0]
    d = g[y0 + 1][:, x0 + 1]
    return a * (1 - fx) * (1 - fy) + b * fx * (1 - fy) + c * (1 - fx) * fy + d * fx * fy


def _gauss1d(sigma):
    r = int(np.ceil(3 * sigma))
    x = np.arange(-r, r + 1, dtype=np.float32)
    k = np.exp(-0.5 * (x / sigma) ** 2)
    return k / k.sum()


def synth_frame(width: int, height: int, seed: int, n_shapes: int = 400) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = 60 * _value_noise(rng, height, width, 48) + 40 * _value_noise(rng, height, width, 12) + 70
    yy, xx = np.mgrid[0:height, 0:width]
    for _ in range(n_shapes):
        val = rng.uniform(0, 255)
        if rng.uniform() < 0.5:
            x0, y0 = rng.integers(0, width), rng.integers(0, height)
            w, h = rng.integers(4, 60), rng.integers(4, 60)
            img[y0:y0 + h, x0:x0 + w] = val
        else:
            cx, cy, r = rng.uniform(0, width), rng.uniform(0, height), rng.uniform(3, 30)
            x0, x1 = max(int(cx - r), 0), min(int(cx + r) + 1, width)
            y0, y1 = max(int(cy - r), 0), min(int(cy + r) + 1, height)
            if x0 >= x1 or y0 >= y1:
                continue
            sub = (xx[y0:y1, x0:x1] - cx) ** 2 + (yy[y0:y1, x0:x1] - cy) ** 2 <= r * r
            img[y0:y1, x0:x1][sub] = val
    k = _gauss1d(0.8)
    img = np.apply_along_axis(lambda r: np.convolve(r, k, mode="same"), 1, img)
    img = np.apply_along_axis(lambda c: np.convolve(c, k, mode="same"), 0, img)
    img += rng.uniform(-3, 3, img.shape)
    return np.ascontiguousarray(np.clip(np.rint(img), 0, 255).astype(np.uint8))


def synth_sequence(camera: str, nframes: int, stream: int = 0) -> np.ndarray:
    w, h = CAMERAS[camera][:2]
    return np.stack([synth_frame(w, h, frame_seed(stream, f)) for f in range(nframes)])


# ----------------------------------------------------------------- scenes
def look_pose(rng, trans_sigma=0.0, rot_deg=0.0) -> np.ndarray:
    """Tcw near identity (camera at the origin looking along +z)."""
    T = np.eye(4)
    if rot_deg:
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        ang = np.radians(rot_deg)
        K = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
        T[:3, :3] = np.eye(3) + np.sin(ang) * K + (1 - np.cos(ang)) * K @ K
    T[:3, 3] = rng.normal(scale=trans_sigma, size=3) if trans_sigma else 0
    return T.astype(np.float32)


def project(T, X, cam):
    w, h, fx, fy, cx, cy = cam
    Pc = X @ T[:3, :3].T.astype(np.float64) + T[:3, 3]
    u = fx * Pc[:, 0] / Pc[:, 2] + cx
    v = fy * Pc[:, 1] / Pc[:, 2] + cy
    return u, v, Pc[:, 2]


def flip_bits(rng, desc, kmax):
    out = desc.copy()
    for i in range(len(out)):
        k = int(rng.integers(0, kmax + 1))
        if k:
            bits = rng.choice(256, k, replace=False)
            for b in bits:
                out[i, b >> 3] ^= np.uint8(1 << (b & 7))
    return out


def synth_scene(camera: str, n_mp: int, n_kp: int, seed: int, nlevels: int = 8, scale: float = 1.2,
                max_flip: int = 40, outlier_frac: float = 0.1):
    """Map points + a frame that observes them.

    Returns dict with map (MAP_POINT_DTYPE), mp_desc, Tcw, keypoints
    (KEYPOINT_DTYPE), descriptors and kp_mp (ground-truth map point per
    keypoint, -1 for distractors)."""
    from .matcher import MAP_POINT_DTYPE
    from .orb import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    cam = CAMERAS[camera]
    w, h = cam[:2]
    X = np.stack([rng.uniform(-4, 4, n_mp), rng.uniform(-3, 3, n_mp), rng.uniform(2, 8, n_mp)], 1)
    Tcw = look_pose(rng, 0.02, 0.5)
    Ow = -(Tcw[:3, :3].T @ Tcw[:3, 3])
    dist = np.linalg.norm(X - Ow, axis=1)
    level = rng.integers(0, nlevels, n_mp)
    sf = np.array([np.float32(scale) ** i for i in range(nlevels)], np.float64)
    mp = np.zeros(n_mp, MAP_POINT_DTYPE)
    mp["pos"] = X
    nrm = (X - Ow) / dist[:, None]
    nrm += rng.normal(scale=0.02, size=nrm.shape)
    mp["normal"] = nrm / np.linalg.norm(nrm, axis=1, keepdims=True)
    # choose min distance so that the predicted level is `level`
    mp["min_dist"] = dist / (sf[level] * 0.97)
    mp["max_dist"] = mp["min_dist"] * sf[-1] * 1.2
    mp_desc = rng.integers(0, 256, (n_mp, 32), dtype=np.uint8)
    u, v, z = project(Tcw, X, cam)
    vis = np.nonzero((z > 0) & (u >= 0) & (u < w) & (v >= 0) & (v < h))[0]
    vis = vis[: n_kp]
    nvis = len(vis)
    kps = np.zeros(n_kp, KEYPOINT_DTYPE)
    kp_mp = np.full(n_kp, -1, np.int32)
    ku = u[vis] + rng.uniform(-1, 1, nvis)
    kv = v[vis] + rng.uniform(-1, 1, nvis)
    nout = int(outlier_frac * nvis)
    sel = rng.choice(nvis, nout, replace=False) if nout else np.zeros(0, int)
    ang = rng.uniform(0, 2 * np.pi, nout)
    rad = rng.uniform(3, 6, nout)
    ku[sel] += rad * np.cos(ang)
    kv[sel] += rad * np.sin(ang)
    kps["x"][:nvis], kps["y"][:nvis] = np.clip(ku, 0, w - 1), np.clip(kv, 0, h - 1)
    lvl = level[vis] - (rng.uniform(size=nvis) < 0.3)
    kps["octave"][:nvis] = np.clip(lvl, 0, nlevels - 1)
    kp_mp[:nvis] = vis
    desc = np.zeros((n_kp, 32), np.uint8)
    desc[:nvis] = flip_bits(rng, mp_desc[vis], max_flip)
    nd = n_kp - nvis
    kps["x"][nvis:] = rng.uniform(0, w - 1, nd)
    kps["y"][nvis:] = rng.uniform(0, h - 1, nd)
    kps["octave"][nvis:] = rng.integers(0, nlevels, nd)
    desc[nvis:] = rng.integers(0, 256, (nd, 32), dtype=np.uint8)
    kps["angle"] = rng.uniform(0, 360, n_kp)
    kps["size"] = 31 * sf[kps["octave"]]
    kps["response"] = rng.integers(7, 80, n_kp)
    kps["class_id"] = -1
    perm = rng.permutation(n_kp)
    kps, desc, kp_mp = kps[perm], desc[perm], kp_mp[perm]
    # level-major order like the extractor output
    order = np.argsort(kps["octave"], kind="stable")
    kps, desc, kp_mp = kps[order], desc[order], kp_mp[order]
    return {"map": mp, "mp_desc": mp_desc, "Tcw": Tcw, "keypoints": np.ascontiguousarray(kps),
            "descriptors": np.ascontiguousarray(desc), "kp_mp": kp_mp, "camera": cam}


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
    from .matcher import MAP_POINT_DTYPE

    mp = np.zeros(n_map, MAP_POINT_DTYPE)
    mp["pos"] = X
    nrm = X / dist[:, None] + rng.normal(scale=0.01, size=X.shape)
    mp["normal"] = nrm / np.linalg.norm(nrm, axis=1, keepdims=True)
    mp["min_dist"] = dist / (sf[lvl] * 0.98)
    mp["max_dist"] = mp["min_dist"] * sf[-1] * 1.2
    mdesc = np.concatenate([flip_bits(rng, desc[sel], max_flip),
                            rng.integers(0, 256, (nd, 32), dtype=np.uint8)])
    perm = rng.permutation(n_map)  # local-map order is arbitrary (Tracking.cc:3780-3821)
    if not return_assoc:
        return mp[perm], np.ascontiguousarray(mdesc[perm])
    inv = np.empty(n_map, np.int64)
    inv[perm] = np.arange(n_map)
    assoc = np.full(n, -1, np.int32)
    assoc[sel] = inv[np.arange(len(sel))]
    return mp[perm], np.ascontiguousarray(mdesc[perm]), assoc


POSE_EDGE_DTYPE = np.dtype([("X", "<f4", 3), ("z", "<f4", 2), ("inv_sigma2", "<f4")])


def synth_pose_problem(seed: int, n: int, camera: str = "euroc", noise_px: float = 1.0, outlier_frac: float = 0.1,
                       rot_deg: float = 0.5, trans: float = 0.01, nlevels: int = 8, scale: float = 1.2):
    """One PoseOptimization problem (SURVEY.md §8d config 4 noise model).

    Map points X ~ U([-4,4]x[-4,4]x[2,8]) seen from a random Tcw_true; keypoint
    z = projection + N(0, noise_px), octave U{0..nlevels-1}; outlier_frac of the
    edges displaced 3-6 px (test_RANSAC.cpp:186-188 style). The initial pose is
    Tcw_true perturbed by rot_deg / trans. Returns (Tcw_true, Tcw_init, edges, cam).
    """
    rng = np.random.default_rng(seed)
    cam = CAMERAS[camera]
    w, h, fx, fy, cx, cy = cam
    T_true = look_pose(rng, trans_sigma=0.3, rot_deg=5.0).astype(np.float64)
    Xs, zs = [], []
    while sum(len(x) for x in Xs) < n:
        Pc = np.c_[rng.uniform(-4, 4, 4 * n), rng.uniform(-4, 4, 4 * n), rng.uniform(2, 8, 4 * n)]
        X = (Pc - T_true[:3, 3]) @ T_true[:3, :3]  # world = R^T (Pc - t)
        u, v, d = project(T_true, X, cam)
        ok = (d > 0.1) & (u >= 0) & (u < w) & (v >= 0) & (v < h)
        Xs.append(X[ok])
        zs.append(np.c_[u[ok], v[ok]])
    X = np.concatenate(Xs)[:n]
    z = np.concatenate(zs)[:n] + rng.normal(0, noise_px, (n, 2))
    nout = int(round(outlier_frac * n))
    if nout:
        idx = rng.choice(n, nout, replace=False)
        ang = rng.uniform(0, 2 * np.pi, nout)
        r = rng.uniform(3, 6, nout)
        z[idx] += np.c_[r * np.cos(ang), r * np.sin(ang)]
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(s[-1] * np.float32(scale)))
    s = np.array(s, np.float32)
    invs = (np.float32(1.0) / (s * s)).astype(np.float32)
    edges = np.zeros(n, POSE_EDGE_DTYPE)
    edges["X"] = X
    edges["z"] = z
    edges["inv_sigma2"] = invs[rng.integers(0, nlevels, n)]
    dT = look_pose(rng, trans_sigma=trans, rot_deg=rot_deg).astype(np.float64)
    T_init = (dT @ T_true).astype(np.float32)
    return T_true.astype(np.float32), T_init, edges, cam


def synth_lba_problem(seed: int, nkf: int = 20, npts: int = 3000, nfixed: int = 2, camera: str = "euroc",
                      noise_px: float = 1.0, outlier_frac: float = 0.05, rot_deg: float = 0.5, trans: float = 0.01,
                      pt_noise: float = 0.02, min_obs: int = 2, max_obs: int = 8, nlevels: int = 8,
                      scale: float = 1.2) -> dict:
    """One LocalBundleAdjustment window.

    nkf local keyframes on a 1 m arc (keyframe 0 is the fixed mnId == 0 one),
    plus nfixed fixed observer cameras (lFixedCameras). npts map points with
    X ~ U([-4,4] x [-4,4] x [2,8]), each observed by U{min_obs..max_obs} of the
    keyframes that see it (observation order per point random, as the
    reference's map<KeyFrame*, size_t> pointer order); z = projection +
    N(0, noise_px), octave U{0..nlevels-1}; outlier_frac of the observations
    displaced 3-6 px. Initial local poses perturbed by rot_deg / trans, points
    by N(0, pt_noise). Arrays follow gf_ba_problem (include/gfslam/abi.h)."""
    rng = np.random.default_rng(seed)
    w, h, fx, fy, cx, cy = CAMERAS[camera]
    K = nkf + nfixed
    ang = np.linspace(-0.25, 0.25, K) + rng.normal(0, 0.01, K)
    centers = np.c_[2 * np.sin(ang), rng.normal(0, 0.05, K), 2 - 2 * np.cos(ang)]
    T_true = np.zeros((K, 4, 4))
    for k in range(K):
        c, s = np.cos(-ang[k] * 0.5), np.sin(-ang[k] * 0.5)
        R = np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
        T_true[k] = np.eye(4)
        T_true[k, :3, :3] = R
        T_true[k, :3, 3] = -R @ centers[k]
    kind = np.zeros(K, np.uint8)  # vertex-id order; fixed cameras interleave with the local keyframes
    kind[0] = 1
    kind[rng.choice(np.arange(1, K), nfixed, replace=False)] = 2
    X, obs = [], []
    while len(X) < npts:
        P = np.c_[rng.uniform(-4, 4, 4 * npts), rng.uniform(-4, 4, 4 * npts), rng.uniform(2, 8, 4 * npts)]
        Pc = np.einsum("kij,nj->kni", T_true[:, :3, :3], P) + T_true[:, None, :3, 3]
        u = fx * Pc[..., 0] / Pc[..., 2] + cx
        v = fy * Pc[..., 1] / Pc[..., 2] + cy
        vis = (Pc[..., 2] > 0.1) & (u >= 0) & (u < w) & (v >= 0) & (v < h)
        for i in np.nonzero(vis.sum(0) >= min_obs)[0]:
            ks = np.nonzero(vis[:, i])[0]
            m = int(rng.integers(min_obs, min(max_obs, len(ks)) + 1))
            sel = rng.permutation(rng.choice(ks, m, replace=False))
            X.append(P[i])
            obs.append([(int(k), u[k, i], v[k, i]) for k in sel])
            if len(X) == npts:
                break
    X = np.array(X)
    e_pt = np.array([i for i, o in enumerate(obs) for _ in o], np.int32)
    e_kf = np.array([k for o in obs for (k, _, _) in o], np.int32)
    z = np.array([(uu, vv) for o in obs for (_, uu, vv) in o]) + rng.normal(0, noise_px, (len(e_pt), 2))
    nout = int(round(outlier_frac * len(e_pt)))
    if nout:
        idx = rng.choice(len(e_pt), nout, replace=False)
        a = rng.uniform(0, 2 * np.pi, nout)
        r = rng.uniform(3, 6, nout)
        z[idx] += np.c_[r * np.cos(a), r * np.sin(a)]
    s = [np.float32(1.0)]
    for _ in range(1, nlevels):
        s.append(np.float32(s[-1] * np.float32(scale)))
    s = np.array(s, np.float32)
    invs = (np.float32(1.0) / (s * s)).astype(np.float32)
    T0 = T_true.copy()
    for k in range(K):
        if kind[k] == 0:
            T0[k] = look_pose(rng, trans, rot_deg).astype(np.float64) @ T_true[k]
    X0 = X + rng.normal(0, pt_noise, X.shape)
    return {"kf_Tcw": np.ascontiguousarray(T0.reshape(K, 16), np.float32), "kf_kind": kind,
            "kf_cam": np.tile(np.array([fx, fy, cx, cy], np.float32), (K, 1)),
            "pt_pos": np.ascontiguousarray(X0, np.float32), "edge_pt": e_pt, "edge_kf": e_kf,
            "edge_z": np.ascontiguousarray(z, np.float32),
            "edge_inv_sigma2": invs[rng.integers(0, nlevels, len(e_pt))],
            "T_true": T_true.astype(np.float32), "X_true": X.astype(np.float32)}


def synth_vocabulary(seed: int = 7, k: int = 10, L: int = 3, flip: int = 40, stop_frac: float = 0.02,
                     scoring: int = 0, weighting: int = 0) -> dict:
    """A k-ary, L-level ORB vocabulary tree in the loaders' node order (SURVEY.md
    §8d: random-descriptor tree, seed 7): breadth first, so a node's children
    are consecutive records. Level-1 descriptors are random; a child is its
    parent with `flip` random bits flipped, so descents are informative.
    Leaves carry idf-like weights in [0.5, 5) with `stop_frac` stopped (0)."""
    rng = np.random.default_rng(seed)
    parent, desc, leaf = [-1], [np.zeros(32, np.uint8)], [0]
    level = [0]
    for lev in range(1, L + 1):
        nxt = []
        for p in level:
            base = desc[p] if lev > 1 else None
            for _ in range(k):
                if base is None:
                    d = rng.integers(0, 256, 32, dtype=np.uint8)
                else:
                    d = flip_bits(rng, base[None], flip)[0] if flip else base.copy()
                parent.append(p)
                desc.append(d)
                leaf.append(1 if lev == L else 0)
                nxt.append(len(parent) - 1)
        level = nxt
    n = len(parent)
    weight = np.zeros(n)
    lv = np.array(leaf, bool)
    weight[lv] = rng.uniform(0.5, 5.0, lv.sum())
    weight[lv & (rng.uniform(size=n) < stop_frac)] = 0.0
    return {"k": k, "L": L, "scoring": scoring, "weighting": weighting, "parent": np.array(parent, np.int32),
            "desc": np.ascontiguousarray(np.stack(desc), np.uint8), "weight": weight, "is_leaf": lv.astype(np.uint8)}


def synth_vocabulary_fast(seed: int = 7, k: int = 10, L: int = 6, stop_frac: float = 0.02) -> dict:
    """ORBvoc-sized tree (k = 10, L = 6: 1,111,111 nodes, ~50 MB) in the loaders'
    breadth-first node order, vectorised level by level: a child is its parent
    with each bit flipped with probability 1/8 (AND of three random bytes).
    Used for the start-up vocabulary broadcast (bench.py); the tests use the
    smaller synth_vocabulary."""
    rng = np.random.default_rng(seed)
    descs = [np.zeros((1, 32), np.uint8)]
    parents = [np.array([-1], np.int32)]
    first = 0  # node id of the first node of the previous level
    for lev in range(1, L + 1):
        prev = descs[-1]
        n = len(prev) * k
        if lev == 1:
            d = rng.integers(0, 256, (n, 32), dtype=np.uint8)
        else:
            m = rng.integers(0, 256, (3, n, 32), dtype=np.uint8)
            d = np.repeat(prev, k, axis=0) ^ (m[0] & m[1] & m[2])
        descs.append(d)
        parents.append((first + np.arange(len(prev), dtype=np.int32)).repeat(k))
        first += len(prev)
    parent = np.concatenate(parents)
    nn = len(parent)
    leaf = np.zeros(nn, np.uint8)
    leaf[nn - k ** L:] = 1
    weight = np.zeros(nn)
    weight[nn - k ** L:] = rng.uniform(0.5, 5.0, k ** L)
    weight[(leaf == 1) & (rng.uniform(size=nn) < stop_frac)] = 0.0
    return {"k": k, "L": L, "scoring": 0, "weighting": 0, "parent": parent,
            "desc": np.ascontiguousarray(np.concatenate(descs)), "weight": weight, "is_leaf": leaf}


def pack_vocabulary(voc: dict) -> np.ndarray:
    """One byte blob: int32 header (k, L, scoring, weighting, nnodes, 0), then
    parent i32, descriptors 32 B, weights f64, is_leaf u8."""
    n = len(voc["parent"])
    hdr = np.array([voc["k"], voc["L"], voc["scoring"], voc["weighting"], n, 0], np.int32)
    return np.concatenate([hdr.view(np.uint8), voc["parent"].astype(np.int32).view(np.uint8),
                           voc["desc"].reshape(-1), voc["weight"].astype(np.float64).view(np.uint8),
                           voc["is_leaf"].astype(np.uint8)])


def unpack_vocabulary(blob: np.ndarray) -> dict:
    hdr = blob[:24].view(np.int32)
    n = int(hdr[4])
    o = 24
    parent = blob[o:o + 4 * n].view(np.int32); o += 4 * n
    desc = blob[o:o + 32 * n].reshape(n, 32); o += 32 * n
    weight = blob[o:o + 8 * n].view(np.float64); o += 8 * n
    leaf = blob[o:o + n]
    return {"k": int(hdr[0]), "L": int(hdr[1]), "scoring": int(hdr[2]), "weighting": int(hdr[3]),
            "parent": parent.copy(), "desc": desc.copy(), "weight": weight.copy(), "is_leaf": leaf.copy()}


def vocab_features(voc: dict, n: int, seed: int, flip: int = 20) -> np.ndarray:
    """Descriptors drawn near random leaves of the vocabulary (a frame's ORB
    features), so FeatureVector nodes hold several features."""
    rng = np.random.default_rng(seed)
    leaves = np.nonzero(voc["is_leaf"])[0]
    src = voc["desc"][rng.choice(leaves, n)]
    return np.ascontiguousarray(flip_bits(rng, src, flip))


def write_vocab_binary(voc: dict, path: str) -> None:
    """TemplatedVocabulary::saveToBinaryFile layout (TemplatedVocabulary.h:1516-1536)."""
    n = len(voc["parent"])
    rec = np.zeros(n - 1, np.dtype([("parent", "<i4"), ("desc", "u1", 32), ("weight", "<f4"), ("leaf", "u1")]))
    rec["parent"] = voc["parent"][1:]
    rec["desc"] = voc["desc"][1:]
    rec["weight"] = voc["weight"][1:]
    rec["leaf"] = voc["is_leaf"][1:]
    with open(path, "wb") as f:
        f.write(np.array([n, 41], "<u4").tobytes())
        f.write(np.array([voc["k"], voc["L"], voc["scoring"], voc["weighting"]], "<i4").tobytes())
        f.write(rec.tobytes())


def write_vocab_text(voc: dict, path: str) -> None:
    """TemplatedVocabulary::saveToTextFile layout (TemplatedVocabulary.h:1443-1462)."""
    with open(path, "w") as f:
        f.write(f"{voc['k']} {voc['L']}  {voc['scoring']} {voc['weighting']}\n")
        for i in range(1, len(voc["parent"])):
            d = " ".join(str(int(x)) for x in voc["desc"][i])
            f.write(f"{voc['parent'][i]} {int(voc['is_leaf'][i])} {d}  {float(voc['weight'][i])!r}\n")


def synth_covis_graph(seed: int, nkf: int = 300, nmp: int = 20000, slots: int = 1000, bad_kf: float = 0.05,
                      bad_mp: float = 0.05, span: int = 6, max_obs: int = 8) -> dict:
    """A map for local-map assembly (localmap.CovisGraph):
    nkf keyframes along a trajectory, each map point observed by 2..max_obs
    keyframes within `span` of its home keyframe (one slot each, slots
    shuffled, the rest NULL), covisibility = keyframes sharing points ordered
    by shared count (descending, then index) as UpdateBestCovisibles does;
    a fraction of keyframes and points is bad."""
    rng = np.random.default_rng(seed)
    home = np.sort(rng.integers(0, nkf, nmp))
    obs = []
    for m in range(nmp):
        k = int(rng.integers(2, max_obs + 1))
        lo, hi = max(0, home[m] - span), min(nkf, home[m] + span + 1)
        obs.append(np.sort(rng.choice(np.arange(lo, hi), size=min(k, hi - lo), replace=False)))
    kf_slots = [[] for _ in range(nkf)]
    for m, o in enumerate(obs):
        for k in o:
            kf_slots[k].append(m)
    kf_mp_off = [0]
    kf_mp = []
    for k in range(nkf):
        s = np.full(max(slots, len(kf_slots[k])), -1, np.int32)
        pos = rng.choice(len(s), size=len(kf_slots[k]), replace=False)
        s[pos] = kf_slots[k]
        kf_mp.append(s)
        kf_mp_off.append(kf_mp_off[-1] + len(s))
    shared = np.zeros((nkf, nkf), np.int32)
    for o in obs:
        for a in o:
            for b in o:
                if a != b:
                    shared[a, b] += 1
    kf_cov_off = [0]
    kf_cov = []
    for k in range(nkf):
        nb = np.nonzero(shared[k] >= 15)[0]
        nb = nb[np.lexsort((nb, -shared[k, nb]))]
        kf_cov.append(nb.astype(np.int32))
        kf_cov_off.append(kf_cov_off[-1] + len(nb))
    mp_obs_off = np.concatenate([[0], np.cumsum([len(o) for o in obs])]).astype(np.int32)
    return dict(kf_bad=(rng.random(nkf) < bad_kf).astype(np.uint8), kf_mp_off=np.array(kf_mp_off, np.int32),
                kf_mp=np.concatenate(kf_mp) if kf_mp else np.zeros(0, np.int32),
                kf_cov_off=np.array(kf_cov_off, np.int32),
                kf_cov=np.concatenate(kf_cov) if kf_cov else np.zeros(0, np.int32),
                mp_bad=(rng.random(nmp) < bad_mp).astype(np.uint8), mp_obs_off=mp_obs_off,
                mp_obs=np.concatenate(obs).astype(np.int32) if obs else np.zeros(0, np.int32))


def synth_frame_mps(seed: int, graph: dict, nkp: int = 1000, center: int | None = None, matched: float = 0.4,
                    window: int = 4) -> np.ndarray:
    """mvpMapPoints of a frame near keyframe `center`: a fraction of the
    keypoints matched to points observed by keyframes within `window`
    (duplicates possible, bad points included as the reference's frame may
    hold them), the rest NULL."""
    rng = np.random.default_rng(seed)
    nkf = len(graph["kf_bad"])
    c = int(rng.integers(0, nkf)) if center is None else center
    lo, hi = max(0, c - window), min(nkf, c + window + 1)
    cand = graph["kf_mp"][graph["kf_mp_off"][lo]:graph["kf_mp_off"][hi]]
    cand = cand[cand >= 0]
    fm = np.full(nkp, -1, np.int32)
    if len(cand):
        on = rng.random(nkp) < matched
        fm[on] = rng.choice(cand, size=int(on.sum()))
    return fm


def synth_two_view(seed: int, n_match: int = 300, n_extra: int = 200, planar: bool = False, baseline: float = 0.3,
                   rot_deg: float = 5.0, noise_px: float = 0.5, outlier_frac: float = 0.1, width: int = 752,
                   height: int = 480, f: float = 458.0) -> dict:
    """Two views of one scene for the monocular initialiser (Initializer.cc):
    reference keypoints kps1, current keypoints kps2 (KEYPOINT_DTYPE, both
    with unmatched extras, shuffled), matches12 (n1 entries, -1 = unmatched),
    K (3x3), and the ground truth R21, t21 (x2 = R21 x1 + t21) and X (points
    in camera-1 coordinates, NaN for outlier matches). planar: the points lie
    on one plane (the homography case); baseline 0 is a pure rotation (no
    parallax: the initialisation has to fail)."""
    from .orb import KEYPOINT_DTYPE
    rng = np.random.default_rng(seed)
    K = np.array([[f, 0, width / 2], [0, f, height / 2], [0, 0, 1]], np.float32)
    ax = rng.normal(size=3)
    ax /= np.linalg.norm(ax)
    a = np.deg2rad(rot_deg)
    S = np.array([[0, -ax[2], ax[1]], [ax[2], 0, -ax[0]], [-ax[1], ax[0], 0]])
    R = np.eye(3) + np.sin(a) * S + (1 - np.cos(a)) * S @ S
    tdir = rng.normal(size=3) * [1.0, 0.3, 0.2]
    t = baseline * tdir / max(np.linalg.norm(tdir), 1e-12)

    def project(P):
        return (P[:, :2] / P[:, 2:3]) * [K[0, 0], K[1, 1]] + [K[0, 2], K[1, 2]]

    X = np.zeros((0, 3))
    while len(X) < n_match:
        m = 4 * n_match
        uv = rng.uniform([20, 20], [width - 20, height - 20], size=(m, 2))
        if planar:
            nrm = np.array([0.1, -0.2, 1.0]) + 0.1 * rng.normal(size=3)
            d = 4.0
            ray = np.c_[(uv - K[:2, 2]) / [K[0, 0], K[1, 1]], np.ones(m)]
            z = d / (ray @ nrm)
            P = ray * z[:, None]
        else:
            z = rng.uniform(2.0, 8.0, size=m)
            P = np.c_[(uv - K[:2, 2]) / [K[0, 0], K[1, 1]] * z[:, None], z]
        P2 = P @ R.T + t
        u2 = project(P2) if len(P2) else P2[:, :2]
        ok = (P[:, 2] > 0.5) & (P2[:, 2] > 0.5) & (u2[:, 0] > 5) & (u2[:, 0] < width - 5) & (u2[:, 1] > 5) & \
             (u2[:, 1] < height - 5)
        X = np.r_[X, P[ok]]
    X = X[:n_match]
    u1 = project(X) + rng.normal(scale=noise_px, size=(n_match, 2))
    u2 = project(X @ R.T + t) + rng.normal(scale=noise_px, size=(n_match, 2))
    nout = int(round(outlier_frac * n_match))
    out_idx = rng.choice(n_match, nout, replace=False)
    u2[out_idx] = rng.uniform([5, 5], [width - 5, height - 5], size=(nout, 2))
    Xgt = X.copy()
    Xgt[out_idx] = np.nan
    n1, n2 = n_match + n_extra, n_match + n_extra

    def kparr(uv):
        k = np.zeros(len(uv), KEYPOINT_DTYPE)
        k["x"], k["y"] = uv[:, 0], uv[:, 1]
        k["size"] = 31.0
        k["angle"] = rng.uniform(0, 360, size=len(uv))
        k["response"] = rng.uniform(0, 100, size=len(uv))
        k["octave"] = rng.integers(0, 4, size=len(uv))
        k["class_id"] = -1
        return k

    e1 = rng.uniform([5, 5], [width - 5, height - 5], size=(n_extra, 2))
    e2 = rng.uniform([5, 5], [width - 5, height - 5], size=(n_extra, 2))
    p1, p2 = rng.permutation(n1), rng.permutation(n2)  # keypoint order in each frame
    kps1 = kparr(np.r_[u1, e1])[np.argsort(p1)]
    kps2 = kparr(np.r_[u2, e2])[np.argsort(p2)]
    # row r of the stacked arrays sits at position p[r]
    matches12 = np.full(n1, -1, np.int32)
    matches12[p1[:n_match]] = p2[:n_match]
    X1 = np.full((n1, 3), np.nan)
    X1[p1[:n_match]] = Xgt
    return dict(kps1=kps1, kps2=kps2, matches12=matches12, K=K, R21=R.astype(np.float32), t21=t.astype(np.float32),
                X=X1)
