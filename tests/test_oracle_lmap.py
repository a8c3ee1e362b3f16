"""Pins the CPU oracle's local-mapping rows against
independent pure-Python restatements of the reference loops on small cases:
MapPoint::ComputeDistinctiveDescriptors (MapPoint.cc:227-261), ORBmatcher::
Fuse (ORBmatcher.cc:1590-1707) and SearchForTriangulation (:1426-1588). The
reference ships no test or fixture for these functions, so parity is pinned
restatement-to-restatement (noted in DESIGN.md)."""
import math

import numpy as np
import pytest

import lmap_scenes as S
import oracle_lib as O
from gf_orb_slam_amd.matcher import FUSE_ADD, FUSE_KEEP, FUSE_NONE, FUSE_REPLACE

f32 = np.float32


def _ham(a, b):
    return int(np.unpackbits(np.bitwise_xor(a, b)).sum())


def _distinctive_py(desc, offs):
    out = []
    for p in range(len(offs) - 1):
        D = desc[offs[p]:offs[p + 1]]
        N = len(D)
        if N == 0:
            out.append(-1)
            continue
        M = np.unpackbits(D[:, None, :] ^ D[None, :, :], axis=2).sum(2)
        med = np.sort(M, 1)[:, int(0.5 * (N - 1))]
        out.append(int(np.argmin(med)))  # first minimum
    return np.array(out, np.int32)


@pytest.mark.parametrize("seed,max_obs", [(1, 12), (2, 40), (3, 3)])
def test_distinctive_oracle_vs_python(seed, max_obs):
    d, off = S.observation_sets(seed, 120, max_obs)
    b, od = O.distinctive_descriptors(d, off)
    assert np.array_equal(b, _distinctive_py(d, off))
    for p in np.nonzero(b >= 0)[0]:
        assert np.array_equal(od[p], d[off[p] + b[p]])


def _cround(x):  # std::round: half away from zero
    return int(math.copysign(math.floor(abs(x) + 0.5), x))


def _fuse_py(info, T, Ow, kps, desc, kf_mp, kf_bad, mps, md, skip, ids, th):
    T = T.astype(f32)
    invW = f32(64) / f32(info.max_x - info.min_x)
    invH = f32(48) / f32(info.max_y - info.min_y)
    grid = [[[] for _ in range(48)] for _ in range(64)]
    for i, k in enumerate(kps):
        px, py = _cround(float((k["x"] - f32(info.min_x)) * invW)), _cround(float((k["y"] - f32(info.min_y)) * invH))
        if 0 <= px < 64 and 0 <= py < 48:
            grid[px][py].append(i)
    scales = [f32(1)]
    for _ in range(1, info.nlevels):
        scales.append(f32(scales[-1] * f32(info.scale_factor)))
    occ, bad = list(kf_mp), list(kf_bad)
    res, nf = [], 0
    for i, mp in enumerate(mps):
        r = [-1, FUSE_NONE, -1]
        res.append(r)
        if skip[i]:
            continue
        P = mp["pos"]
        Pc = [((T[j, 0] * P[0] + T[j, 1] * P[1]) + T[j, 2] * P[2]) + T[j, 3] for j in range(3)]
        if Pc[2] < f32(0):
            continue
        invz = f32(1) / Pc[2]
        x, y = Pc[0] * invz, Pc[1] * invz
        u, v = f32(info.fx) * x + f32(info.cx), f32(info.fy) * y + f32(info.cy)
        if not (u >= info.min_x and u < info.max_x and v >= info.min_y and v < info.max_y):
            continue
        PO = [P[j] - Ow[j] for j in range(3)]
        dist = f32(math.sqrt(sum(float(c) * float(c) for c in PO)))
        if dist < mp["min_dist"] or dist > mp["max_dist"]:
            continue
        if sum(float(PO[j]) * float(mp["normal"][j]) for j in range(3)) < 0.5 * float(dist):
            continue
        ratio = dist / mp["min_dist"]
        lvl = min(next((l for l, s in enumerate(scales) if not s < ratio), len(scales)), info.nlevels - 1)
        rad = f32(th) * scales[lvl]
        x0 = max(0, math.floor((u - f32(info.min_x) - rad) * invW))
        x1 = min(63, math.ceil((u - f32(info.min_x) + rad) * invW))
        y0 = max(0, math.floor((v - f32(info.min_y) - rad) * invH))
        y1 = min(47, math.ceil((v - f32(info.min_y) + rad) * invH))
        if x0 >= 64 or x1 < 0 or y0 >= 48 or y1 < 0:
            continue
        best, bi = 1 << 30, -1
        for cx in range(x0, x1 + 1):
            for cy in range(y0, y1 + 1):
                for idx in grid[cx][cy]:
                    k = kps[idx]
                    if abs(k["x"] - u) > rad or abs(k["y"] - v) > rad:
                        continue
                    if k["octave"] < lvl - 1 or k["octave"] > lvl:
                        continue
                    d = _ham(md[i], desc[idx])
                    if d < best:
                        best, bi = d, idx
        if best <= 50:
            nf += 1
            r[0] = bi
            if occ[bi] >= 0:
                if bad[bi]:
                    r[1] = FUSE_KEEP
                else:
                    r[1], r[2] = FUSE_REPLACE, occ[bi]
            else:
                r[1] = FUSE_ADD
                occ[bi] = ids[i]
    return nf, np.array(res, np.int32).reshape(-1, 3)


@pytest.mark.parametrize("seed,th", [(1, 3.0), (2, 5.0)])
def test_fuse_oracle_vs_python(seed, th):
    sc = S.fuse_scene(seed, nmp=400, nkp=300, dup=80)
    kf = sc["kf"]
    args = (sc["info"], sc["Tcw"], sc["Ow"], kf.mvKeysUn, kf.mDescriptors, sc["kf_mp"], sc["kf_bad"], sc["mps"],
            sc["mp_desc"], sc["skip"], sc["ids"], th)
    n, r = O.fuse(*args)
    npy, rpy = _fuse_py(*args)
    assert n == npy and n > 20
    assert np.array_equal(np.stack([r["kp"], r["action"], r["target"]], 1), rpy)
    acts = np.bincount(r["action"], minlength=4)
    assert acts[FUSE_ADD] > 0 and acts[FUSE_REPLACE] > 0


def _tri_py(check_ori, a, b, F, s2):
    (fa, da, ka, ma), (fb, db, kb, mb) = a, b
    F = F.reshape(3, 3).astype(f32)
    out = np.full(len(da), -1, np.int32)
    matched = np.zeros(len(db), bool)
    hist = [[] for _ in range(30)]
    bnode = {int(nd): i for i, nd in enumerate(fb.nodes)}
    for ia, nd in enumerate(fa.nodes):  # the merge walk visits exactly the common nodes, in order
        ib = bnode.get(int(nd))
        if ib is None:
            continue
        for i1 in fa.feats[fa.start[ia]:fa.start[ia + 1]]:
            if ma[i1] >= 0:
                continue
            cand = []
            for i2 in fb.feats[fb.start[ib]:fb.start[ib + 1]]:
                if matched[i2] or mb[i2] >= 0:
                    continue
                d = _ham(da[i1], db[i2])
                if d <= 50:
                    cand.append((d, int(i2)))
            if not cand:
                continue
            cand.sort()
            th = 2 * cand[0][0]
            for d, i2 in cand:
                if d > th:
                    break
                k1, k2 = ka[i1], kb[i2]
                la = (k1["x"] * F[0, 0] + k1["y"] * F[1, 0]) + F[2, 0]
                lb = (k1["x"] * F[0, 1] + k1["y"] * F[1, 1]) + F[2, 1]
                lc = (k1["x"] * F[0, 2] + k1["y"] * F[1, 2]) + F[2, 2]
                num = (la * k2["x"] + lb * k2["y"]) + lc
                den = la * la + lb * lb
                if den == 0 or not float(num * num / den) < 3.84 * float(s2[k2["octave"]]):
                    continue
                matched[i2] = True
                out[i1] = i2
                rot = f32(k1["angle"] - k2["angle"])
                if rot < 0:
                    rot = f32(rot + f32(360))
                bin_ = _cround(float(rot * f32(1 / 30)))
                hist[0 if bin_ == 30 else bin_].append(i1)
                break
    if check_ori:
        sizes = [len(h) for h in hist]
        order = sorted(range(30), key=lambda i: (-sizes[i], i))[:3]
        m1, m2, m3 = (sizes[i] for i in order)
        keep = [order[0] if m1 > 0 else -1, order[1] if m2 > 0 else -1, order[2] if m3 > 0 else -1]
        if m2 < 0.1 * m1:
            keep[1] = keep[2] = -1
        elif m3 < 0.1 * m1:
            keep[2] = -1
        for i in range(30):
            if i not in keep:
                out[hist[i]] = -1
    return int((out >= 0).sum()), out


@pytest.mark.parametrize("seed,ori", [(3, True), (4, False)])
def test_triangulation_oracle_vs_python(seed, ori):
    a, b, F, s2 = S.triangulation_pair(seed, 300, 340)
    tup = lambda s: ((s[0].nodes, s[0].start, s[0].feats),) + s[1:]
    n, out = O.search_triangulation(ori, tup(a), tup(b), F, s2)
    npy, opy = _tri_py(ori, a, b, F, s2)
    assert n == npy and np.array_equal(out, opy) and n > 30
