"""Local-map assembly: Tracking::UpdateReference
(Tracking.cc:3689-3852) — the CPU oracle (oracle/refmap.cpp) against a pure
Python restatement of the same loops, then the device (gf_update_reference,
gf_update_reference_dev) against the oracle: frame map points with bad ones
nulled, local keyframes (order included), the reference keyframe and the
local map points (order included), all exact. No reference test or fixture
covers UpdateReference: parity is pinned restatement-to-restatement
(docs/ORACLE_ASSUMPTIONS.md)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd import synth
from gf_orb_slam_amd.localmap import CovisGraph


def oracle_update(g: CovisGraph, fm, kf_cap=None, mp_cap=None):
    o = O.orc()
    fm = np.array(fm, np.int32, copy=True)
    kf_cap = g.nkf if kf_cap is None else kf_cap
    mp_cap = g.nmp if mp_cap is None else mp_cap
    lk = np.zeros(max(kf_cap, 1), np.int32)
    lm = np.zeros(max(mp_cap, 1), np.int32)
    nk, nm, ref = ctypes.c_int(), ctypes.c_int(), ctypes.c_int32()
    m = g.struct()
    rc = o.orc_update_reference(ctypes.byref(m), O._p(fm), len(fm), O._p(lk), ctypes.byref(nk), kf_cap, O._p(lm),
                                ctypes.byref(nm), mp_cap, ctypes.byref(ref))
    return rc, fm, lk[:min(nk.value, kf_cap)].copy(), lm[:min(nm.value, mp_cap)].copy(), ref.value


def python_update(d: dict, fm):
    """The reference loops once more, in Python (dict in key order)."""
    fm = np.array(fm, np.int32, copy=True)
    counter = {}
    for i, m in enumerate(fm):
        if m < 0:
            continue
        if d["mp_bad"][m]:
            fm[i] = -1
            continue
        for k in d["mp_obs"][d["mp_obs_off"][m]:d["mp_obs_off"][m + 1]]:
            counter[int(k)] = counter.get(int(k), 0) + 1
    mx, kfmax, local, mark = 0, -1, [], set()
    for k in sorted(counter):
        if d["kf_bad"][k]:
            continue
        if counter[k] > mx:
            mx, kfmax = counter[k], k
        local.append(k)
        mark.add(k)
    for p in range(len(local)):
        if len(local) > 80:
            break
        k = local[p]
        for nb in d["kf_cov"][d["kf_cov_off"][k]:d["kf_cov_off"][k + 1]][:10]:
            nb = int(nb)
            if not d["kf_bad"][nb] and nb not in mark:
                local.append(nb)
                mark.add(nb)
                break
    if len(local) > 2 * len(counter):  # (never: one neighbour per original keyframe)
        raise AssertionError
    mps, seen = [], set()
    for k in local:
        for m in d["kf_mp"][d["kf_mp_off"][k]:d["kf_mp_off"][k + 1]]:
            m = int(m)
            if m < 0 or m in seen:
                continue
            if not d["mp_bad"][m]:
                mps.append(m)
                seen.add(m)
    return fm, np.array(local, np.int32), np.array(mps, np.int32), kfmax


def _case(seed, nkf=120, nmp=6000, slots=300, **kw):
    d = synth.synth_covis_graph(seed, nkf=nkf, nmp=nmp, slots=slots)
    fm = synth.synth_frame_mps(seed + 1, d, **kw)
    return d, CovisGraph(**d), fm


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_matches_python_restatement(seed):
    d, g, fm = _case(seed)
    rc, f1, k1, m1, r1 = oracle_update(g, fm)
    f2, k2, m2, r2 = python_update(d, fm)
    assert rc == 0 and r1 == r2
    assert np.array_equal(f1, f2) and np.array_equal(k1, k2) and np.array_equal(m1, m2)
    assert len(k1) > 0 and len(m1) > 0


def test_oracle_caps_and_empty():
    d, g, fm = _case(4)
    rc, *_ = oracle_update(g, fm, kf_cap=1, mp_cap=1)
    assert rc == -3  # GF_ERR_CAP
    rc, f, k, m, r = oracle_update(g, np.full(50, -1, np.int32))
    assert rc == 0 and len(k) == 0 and len(m) == 0 and r == -1




@pytest.mark.gpu
@pytest.mark.parametrize("seed,kw", [(5, {}), (6, {"matched": 0.9, "window": 40}), (7, {"matched": 0.05}),
                                     (8, {"nkp": 2000})])
def test_update_reference_bit_exact(seed, kw):
    from gf_orb_slam_amd.localmap import update_reference

    d, g, fm = _case(seed, nkf=200, nmp=12000, slots=400, **kw)
    rc, f1, k1, m1, r1 = oracle_update(g, fm)
    assert rc == 0
    f2, k2, m2, r2 = update_reference(g, fm)
    assert r1 == r2
    assert np.array_equal(f1, f2) and np.array_equal(k1, k2) and np.array_equal(m1, m2)


@pytest.mark.gpu
def test_update_reference_edges():
    """Empty frame, all-bad points, no keyframes, more than 80 voted keyframes
    (the neighbour loop stops at once), caps exceeded."""
    from gf_orb_slam_amd._lib import GFError
    from gf_orb_slam_amd.localmap import update_reference

    d, g, fm = _case(9, nkf=200, nmp=12000, slots=400, matched=0.95, window=150)
    rc, f1, k1, m1, r1 = oracle_update(g, fm)
    assert len(k1) > 80
    f2, k2, m2, r2 = update_reference(g, fm)
    assert r1 == r2 and np.array_equal(k1, k2) and np.array_equal(m1, m2) and np.array_equal(f1, f2)
    empty = np.full(10, -1, np.int32)
    f2, k2, m2, r2 = update_reference(g, empty)
    assert len(k2) == 0 and len(m2) == 0 and r2 == -1
    dd = dict(d)
    dd["mp_bad"] = np.ones_like(d["mp_bad"])
    gb = CovisGraph(**dd)
    f2, k2, m2, r2 = update_reference(gb, fm)
    assert np.all(f2 == -1) and len(k2) == 0 and r2 == -1
    with pytest.raises(GFError):
        update_reference(g, fm, kf_cap=2, mp_cap=2)


@pytest.mark.gpu
def test_update_reference_batch_dev():
    import torch

    from gf_orb_slam_amd.localmap import update_reference_batch

    d, g, _ = _case(10, nkf=250, nmp=15000, slots=400)
    B, stride = 24, 1200
    fms = np.full((B, stride), -1, np.int32)
    nk = np.zeros(B, np.int32)
    for b in range(B):
        f = synth.synth_frame_mps(100 + b, d, nkp=600 + 25 * b, matched=0.2 + 0.03 * b, window=2 + b)
        fms[b, :len(f)] = f
        nk[b] = len(f)
    dg = g.to_device()
    tfm = torch.from_numpy(fms).cuda()
    lk, nlk, lm, nlm, ref = update_reference_batch(dg, tfm, torch.from_numpy(nk).cuda())
    torch.cuda.synchronize()
    lk, nlk, lm, nlm, ref, tfm = (x.cpu().numpy() for x in (lk, nlk, lm, nlm, ref, tfm))
    for b in range(B):
        rc, f1, k1, m1, r1 = oracle_update(g, fms[b, :nk[b]])
        assert rc == 0 and r1 == ref[b]
        assert np.array_equal(f1, tfm[b, :nk[b]])
        assert nlk[b] == len(k1) and np.array_equal(k1, lk[b, :nlk[b]])
        assert nlm[b] == len(m1) and np.array_equal(m1, lm[b, :nlm[b]])
