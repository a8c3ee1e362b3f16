"""Synthetic inputs for the local-mapping matchers:
observation sets for ComputeDistinctiveDescriptors, a keyframe + candidate
list for Fuse, and a two-keyframe epipolar pair for SearchForTriangulation."""
from __future__ import annotations

import numpy as np

from gf_orb_slam_amd import synth
from gf_orb_slam_amd.matcher import Frame, FrameInfo, camera_center
from gf_orb_slam_amd.orb import KEYPOINT_DTYPE


def observation_sets(seed, nmp, max_obs=40, empty_frac=0.05, flip=30):
    """nmp points with 0..max_obs noisy copies of a base descriptor each (a
    few duplicated rows so that medians tie)."""
    rng = np.random.default_rng(seed)
    counts = rng.integers(1, max_obs + 1, nmp)
    counts[rng.uniform(size=nmp) < empty_frac] = 0
    offs = np.zeros(nmp + 1, np.int32)
    offs[1:] = np.cumsum(counts)
    rows = []
    for c in counts:
        base = rng.integers(0, 256, (1, 32), dtype=np.uint8)
        d = synth.flip_bits(rng, np.repeat(base, c, 0), flip)
        if c > 3:
            d[rng.integers(0, c)] = d[rng.integers(0, c)]
        rows.append(d)
    desc = np.concatenate(rows) if rows else np.zeros((0, 32), np.uint8)
    return np.ascontiguousarray(desc), offs


def fuse_scene(seed, nmp=1500, nkp=1000, cam="euroc", occupied=0.4, dup=200, bad_frac=0.1):
    """A keyframe (the scene frame) whose slots hold some of the map points,
    and a candidate list: every map point (those already in the keyframe are
    skipped) plus `dup` near-duplicates that compete for the same slots."""
    sc = synth.synth_scene(cam, nmp, nkp, seed, max_flip=30)
    info = FrameInfo.make(*sc["camera"])
    rng = np.random.default_rng(seed + 7)
    kf = Frame(sc["keypoints"], sc["descriptors"], info, sc["Tcw"])
    kp_mp = sc["kp_mp"]
    occ = (kp_mp >= 0) & (rng.uniform(size=nkp) < occupied)
    kf_mp = np.where(occ, 100000 + kp_mp, -1).astype(np.int32)
    kf_bad = (occ & (rng.uniform(size=nkp) < bad_frac)).astype(np.uint8)
    in_kf = np.zeros(nmp, bool)
    in_kf[kp_mp[occ]] = True
    src = rng.choice(nmp, dup, replace=False)
    mps = np.concatenate([sc["map"], sc["map"][src]])
    md = np.concatenate([sc["mp_desc"], synth.flip_bits(rng, sc["mp_desc"][src], 6)])
    skip = np.concatenate([in_kf, np.zeros(dup, bool)]).astype(np.uint8)  # duplicates are other points
    skip[rng.uniform(size=len(skip)) < 0.03] = 1  # NULL / bad candidates
    perm = rng.permutation(len(mps))
    ids = (200000 + np.arange(len(mps))).astype(np.int32)
    kf.mvpMapPoints = kf_mp.copy()
    return dict(kf=kf, info=info, Tcw=sc["Tcw"], Ow=camera_center(sc["Tcw"]), kf_mp=kf_mp, kf_bad=kf_bad,
                mps=mps[perm], mp_desc=md[perm], skip=skip[perm], ids=ids)


def _skew(t):
    return np.array([[0, -t[2], t[1]], [t[2], 0, -t[0]], [-t[1], t[0], 0]])


def oracle_fv(voc, desc, levelsup=2):
    """FeatureVector from the CPU oracle's transform."""
    import oracle_lib as O
    from gf_orb_slam_amd.bow import FeatureVector
    return FeatureVector(*O.bow_transform(voc, desc, levelsup)[2])


def triangulation_pair(seed, n1=900, n2=1000, nlevels=8, scale=1.2, mp_frac=0.3, flip=12, fv=oracle_fv):
    """Two keyframes seeing the same 3-D points (baseline ~0.3 m) with their
    FeatureVectors (fv(voc, desc)), F12 (LocalMapping::ComputeF12:
    K1^-T [t12]x R12 K2^-1) and pKF2's level sigma2."""
    rng = np.random.default_rng(seed)
    voc = synth.synth_vocabulary(seed, k=10, L=3)
    w, h, fx, fy, cx, cy = synth.CAMERAS["euroc"]
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float64)
    T1 = np.eye(4)
    T2 = synth.look_pose(rng, 0.3, 3.0).astype(np.float64)
    m = min(n1, n2)
    X = np.stack([rng.uniform(-3, 3, m), rng.uniform(-2, 2, m), rng.uniform(3, 9, m)], 1)

    def proj(T):
        P = X @ T[:3, :3].T + T[:3, 3]
        return np.stack([fx * P[:, 0] / P[:, 2] + cx, fy * P[:, 1] / P[:, 2] + cy], 1)

    u1, u2 = proj(T1), proj(T2)
    d1 = synth.vocab_features(voc, n1, seed + 1, flip=10)
    d2 = np.concatenate([synth.flip_bits(rng, d1[:m], flip), synth.vocab_features(voc, n2 - m, seed + 2)])
    k1, k2 = np.zeros(n1, KEYPOINT_DTYPE), np.zeros(n2, KEYPOINT_DTYPE)
    k1["x"][:m], k1["y"][:m] = u1[:, 0], u1[:, 1]
    k2["x"][:m], k2["y"][:m] = u2[:, 0] + rng.normal(0, 0.7, m), u2[:, 1] + rng.normal(0, 0.7, m)
    for k, n in ((k1, n1), (k2, n2)):
        k["x"][m:], k["y"][m:] = rng.uniform(0, w, n - m), rng.uniform(0, h, n - m)
        k["octave"] = rng.integers(0, nlevels, n)
    k1["angle"] = rng.uniform(0, 360, n1)
    k2["angle"][:m] = (k1["angle"][:m] + rng.normal(15, 6, m)) % 360
    k2["angle"][m:] = rng.uniform(0, 360, n2 - m)
    # distractors: some rows of b copy an a descriptor at a random place
    nd = min(80, n2 - m)
    if nd > 0:
        d2[m:m + nd] = synth.flip_bits(rng, d1[rng.integers(0, m, nd)], flip)
    mp1 = np.where(rng.uniform(size=n1) < mp_frac, np.arange(n1) + 5000, -1).astype(np.int32)
    mp2 = np.where(rng.uniform(size=n2) < mp_frac, np.arange(n2) + 9000, -1).astype(np.int32)
    R12 = T1[:3, :3] @ T2[:3, :3].T
    t12 = -R12 @ T2[:3, 3] + T1[:3, 3]
    F12 = (np.linalg.inv(K).T @ _skew(t12) @ R12 @ np.linalg.inv(K)).astype(np.float32)
    sf = [np.float32(1.0)]
    for _ in range(1, nlevels):
        sf.append(np.float32(sf[-1] * np.float32(scale)))
    sigma2 = np.array([np.float32(s * s) for s in sf], np.float32)
    f1, f2 = fv(voc, d1), fv(voc, d2)
    return (f1, d1, k1, mp1), (f2, d2, k2, mp2), F12, sigma2
