"""GPU parity of the local-mapping matchers with the
CPU oracle: ComputeDistinctiveDescriptors picks, Fuse decisions (keypoint,
action, Replace target, nFused) and SearchForTriangulation match vectors are
bit-exact."""
import ctypes

import numpy as np
import pytest

import lmap_scenes as S
import oracle_lib as O
from gf_orb_slam_amd._lib import check, lib, ptr
from gf_orb_slam_amd.bow import ORBVocabulary
from gf_orb_slam_amd.matcher import (FUSE_ADD, FUSE_KEEP, FUSE_REPLACE, FUSE_RESULT_DTYPE, ORBmatcher,
                                     compute_distinctive_descriptors)
from gf_orb_slam_amd.orb import default_context

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed,nmp,max_obs", [(1, 2000, 12), (2, 500, 64), (3, 300, 300), (4, 50, 700)])
def test_distinctive_descriptors_bit_exact(seed, nmp, max_obs):
    """N up to 700 rows: the LDS-staged (<= 256) and the global-memory path."""
    d, off = S.observation_sets(seed, nmp, max_obs)
    cur = np.full((nmp, 32), 0xAB, np.uint8)
    bg, dg = compute_distinctive_descriptors(d, off, cur)
    bo, do = O.distinctive_descriptors(d, off)
    assert np.array_equal(bg, bo)
    empty = bo < 0
    assert np.array_equal(dg[~empty], do[~empty]) and (dg[empty] == 0xAB).all()


def test_distinctive_descriptors_edges():
    rng = np.random.default_rng(0)
    d = rng.integers(0, 256, (5, 32), dtype=np.uint8)
    off = np.array([0, 0, 1, 3, 3, 5], np.int32)  # empty, single, pair, empty, pair
    bg, _ = compute_distinctive_descriptors(d, off)
    bo, _ = O.distinctive_descriptors(d, off)
    assert np.array_equal(bg, bo) and list(bg) == [-1, 0, 0, -1, 0]
    same = np.repeat(d[:1], 9, 0)  # all ties: first index
    assert compute_distinctive_descriptors(same, np.array([0, 9], np.int32))[0][0] == 0
    assert len(compute_distinctive_descriptors(d[:0], np.zeros(1, np.int32))[0]) == 0


def _fuse_args(sc, th):
    kf = sc["kf"]
    return (sc["info"], sc["Tcw"], sc["Ow"], kf.mvKeysUn, kf.mDescriptors, sc["kf_mp"], sc["kf_bad"], sc["mps"],
            sc["mp_desc"], sc["skip"], sc["ids"], th)


@pytest.mark.parametrize("seed,cam,th", [(1, "euroc", 3.0), (2, "euroc", 5.0), (3, "tum", 3.0), (4, "tum", 1.0)])
def test_fuse_bit_exact(seed, cam, th):
    sc = S.fuse_scene(seed, nmp=3000, nkp=2000 if cam == "tum" else 1000, cam=cam, dup=400)
    n, r = ORBmatcher().Fuse(sc["kf"], sc["Ow"], sc["mps"], sc["mp_desc"], th, sc["kf_bad"], sc["skip"], sc["ids"])
    no, ro = O.fuse(*_fuse_args(sc, th))
    assert n == no and r.tobytes() == ro.tobytes()
    acts = np.bincount(r["action"], minlength=4)
    assert acts[FUSE_ADD] > 0 and acts[FUSE_REPLACE] > 0
    # the keyframe's slots now hold the added candidates
    add = r["action"] == FUSE_ADD
    assert np.array_equal(sc["kf"].mvpMapPoints[r["kp"][add]], sc["ids"][add])


def test_fuse_optional_inputs_and_empty():
    sc = S.fuse_scene(5, nmp=800, nkp=600, dup=100)
    n, r = ORBmatcher().Fuse(sc["kf"], sc["Ow"], sc["mps"], sc["mp_desc"], 3.0)
    no, ro = O.fuse(sc["info"], sc["Tcw"], sc["Ow"], sc["kf"].mvKeysUn, sc["kf"].mDescriptors, sc["kf_mp"], None,
                    sc["mps"], sc["mp_desc"], None, None, 3.0)
    assert n == no and r.tobytes() == ro.tobytes() and not (r["action"] == FUSE_KEEP).any()
    n0, r0 = ORBmatcher().Fuse(sc["kf"], sc["Ow"], sc["mps"][:0], sc["mp_desc"][:0], 3.0)
    assert n0 == 0 and len(r0) == 0


def test_fuse_dev_batch():
    """gf_fuse_dev: several independent (keyframe, candidates) problems in one launch."""
    import torch
    from gf_orb_slam_amd.matcher import FuseProblem
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    scs = [S.fuse_scene(10 + i, nmp=1200, nkp=900, dup=150) for i in range(4)]
    keep, probs, outs = [], [], []
    for sc in scs:
        kf = sc["kf"]
        bufs = [t(kf.mvKeysUn.view(np.uint8)), t(kf.mDescriptors), t(sc["kf_mp"]), t(sc["kf_bad"]),
                t(sc["mps"].view(np.uint8)), t(sc["mp_desc"]), t(sc["skip"]), t(sc["ids"]),
                torch.zeros(len(sc["mps"]) * 3, dtype=torch.int32, device=dev),
                torch.zeros(1, dtype=torch.int32, device=dev)]
        keep += bufs
        outs.append((bufs[8], bufs[9]))
        probs.append(FuseProblem.make(sc["Tcw"], sc["Ow"], bufs, kf.N, len(sc["mps"]), 3.0))
    arr = (FuseProblem * len(probs))(*probs)
    ctx = default_context()
    check(lib().gf_fuse_dev(ctx.handle, ctypes.byref(scs[0]["info"]), len(probs), arr, ctx.stream))
    check(lib().gf_ctx_sync(ctx.handle))
    for sc, (res, nf) in zip(scs, outs):
        no, ro = O.fuse(*_fuse_args(sc, 3.0))
        rg = res.cpu().numpy().view(FUSE_RESULT_DTYPE)
        assert nf.item() == no and rg.tobytes() == ro.tobytes()


def _gpu_fv(voc, desc, levelsup=2):
    return ORBVocabulary(voc).transform(desc, levelsup)[2]


@pytest.mark.parametrize("seed,ori,n1,n2", [(3, True, 900, 1000), (4, False, 900, 1000), (5, True, 2000, 1800),
                                            (6, True, 60, 4000)])
def test_search_for_triangulation_bit_exact(seed, ori, n1, n2):
    a, b, F, s2 = S.triangulation_pair(seed, n1, n2, fv=_gpu_fv)
    ng, og, pairs = ORBmatcher(0.6, ori).SearchForTriangulation(a, b, F, s2)
    tup = lambda s: ((s[0].nodes, s[0].start, s[0].feats),) + s[1:]
    no, oo = O.search_triangulation(ori, tup(a), tup(b), F, s2)
    assert ng == no and np.array_equal(og, oo) and ng > 20
    assert np.array_equal(pairs[:, 1], og[pairs[:, 0]]) and len(pairs) == ng


def test_search_for_triangulation_edges():
    a, b, F, s2 = S.triangulation_pair(7, 200, 220, fv=_gpu_fv)
    tup = lambda s: ((s[0].nodes, s[0].start, s[0].feats),) + s[1:]
    allmp = (b[0], b[1], b[2], np.arange(len(b[1]), dtype=np.int32))  # every b keypoint already has a MapPoint
    ng, og, _ = ORBmatcher().SearchForTriangulation(a, allmp, F, s2)
    assert ng == 0 and (og == -1).all()
    zero = np.zeros((3, 3), np.float32)  # den == 0: CheckDistEpipolarLine rejects
    ng, og, _ = ORBmatcher().SearchForTriangulation(a, b, zero, s2)
    no, oo = O.search_triangulation(True, tup(a), tup(b), zero, s2)
    assert ng == no == 0


def test_search_for_triangulation_dev_batch():
    """gf_search_for_triangulation_dev: the new keyframe against several
    neighbours in one launch (LocalMapping::CreateNewMapPoints' loop)."""
    import torch
    from gf_orb_slam_amd.bow import BowSide
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    keep, sa, sb, outs, Fs, ref = [], [], [], [], [], []
    for seed in range(20, 26):
        a, b, F, s2 = S.triangulation_pair(seed, 700, 800, fv=_gpu_fv)
        for side, lst in ((a, sa), (b, sb)):
            fv, d, k, mp = side
            bufs = [t(fv.nodes), t(fv.start), t(fv.feats), t(d), t(k.view(np.uint8)), t(mp)]
            keep += bufs
            pn, ps, pf, pd, pk, pm = (x.data_ptr() for x in bufs)
            lst.append(BowSide(pn, ps, pf, len(fv.nodes), pd, pk, pm, len(d)))
        o = torch.full((len(a[1]),), -7, dtype=torch.int32, device=dev)
        outs.append(o)
        Fs.append(F.reshape(9))
        tup = lambda s: ((s[0].nodes, s[0].start, s[0].feats),) + s[1:]
        ref.append(O.search_triangulation(True, tup(a), tup(b), F, s2))
    P = len(outs)
    nm = torch.zeros(P, dtype=torch.int32, device=dev)
    Fh = np.ascontiguousarray(np.stack(Fs), np.float32)
    ctx = default_context()
    check(lib().gf_search_for_triangulation_dev(ctx.handle, 1, P, (BowSide * P)(*sa), (BowSide * P)(*sb), ptr(Fh),
                                                ptr(s2), len(s2), (ctypes.c_void_p * P)(*[o.data_ptr() for o in outs]), ptr(nm), ctx.stream))
    check(lib().gf_ctx_sync(ctx.handle))
    for p, (no, oo) in enumerate(ref):
        og = outs[p].cpu().numpy()
        assert nm[p].item() == no and np.array_equal(og, oo)
