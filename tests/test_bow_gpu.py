"""GPU parity of rows D1 (DBoW2 transform) and M6 (SearchByBoW) with the CPU
oracle: word ids, node ids, feature lists, match vectors and counts are
bit-exact; BowVector values too (sums in the oracle's order)."""
import ctypes

import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd._lib import check, lib, ptr
from gf_orb_slam_amd.bow import BowSide, FeatureVector, ORBVocabulary, search_by_bow
from gf_orb_slam_amd.orb import KEYPOINT_DTYPE, default_context
from gf_orb_slam_amd.synth import flip_bits, synth_vocabulary, vocab_features, write_vocab_binary

pytestmark = pytest.mark.gpu


def _same_transform(g, o):
    gw, gv, gf = g
    ow, ov, (on, os_, of) = o
    assert np.array_equal(gw, ow)
    assert np.array_equal(gv, ov), np.abs(gv - ov).max()
    assert np.array_equal(gf.nodes, on) and np.array_equal(gf.start, os_) and np.array_equal(gf.feats, of)


@pytest.mark.parametrize("k,L,scoring,weighting,levelsup,n", [
    (10, 3, 0, 0, 1, 1000), (10, 3, 0, 0, 4, 1000), (8, 4, 1, 1, 2, 2000), (6, 3, 5, 0, 1, 500),
    (6, 3, 5, 2, 1, 500), (5, 3, 3, 3, 2, 4096), (10, 2, 0, 0, 1, 1), (10, 2, 0, 0, 1, 0)])
def test_transform_matches_oracle(k, L, scoring, weighting, levelsup, n):
    voc = synth_vocabulary(11 + k + L, k=k, L=L, scoring=scoring, weighting=weighting, stop_frac=0.05)
    d = vocab_features(voc, n, 5) if n else np.zeros((0, 32), np.uint8)
    V = ORBVocabulary(voc)
    _same_transform(V.transform(d, levelsup), O.bow_transform(voc, d, levelsup))


def test_vocab_file_and_dev_batch(tmp_path):
    voc = synth_vocabulary(7, k=10, L=3)
    p = str(tmp_path / "voc.bin")
    write_vocab_binary(voc, p)
    V = ORBVocabulary(path=p)
    info = V.info()
    assert info["nnodes"] == len(voc["parent"]) + 1 and info["nwords"] == int(voc["is_leaf"].sum()) + 1
    from gf_orb_slam_amd.bow import read_vocabulary
    tree = read_vocabulary(p)
    import torch
    F, cap = 5, 1200
    descs = [vocab_features(voc, n, 30 + i) for i, n in enumerate([1000, 1200, 7, 0, 640])]
    D = np.zeros((F, cap, 32), np.uint8)
    N = np.array([len(x) for x in descs], np.int32)
    for i, x in enumerate(descs):
        D[i, :len(x)] = x
    dev = torch.device("cuda:0")
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    dD, dN = t(D), t(N)
    w = torch.zeros(F, cap, dtype=torch.int32, device=dev)
    v = torch.zeros(F, cap, dtype=torch.float64, device=dev)
    nw = torch.zeros(F, dtype=torch.int32, device=dev)
    nodes = torch.zeros(F, cap, dtype=torch.int32, device=dev)
    start = torch.zeros(F, cap + 1, dtype=torch.int32, device=dev)
    feats = torch.zeros(F, cap, dtype=torch.int32, device=dev)
    nf = torch.zeros(F, dtype=torch.int32, device=dev)
    ctx = default_context()
    check(lib().gf_bow_transform_dev(V.handle, F, ptr(dD), ptr(dN), cap, 1, ptr(w), ptr(v), ptr(nw), ptr(nodes),
                                     ptr(start), ptr(feats), ptr(nf), ctx.stream))
    check(lib().gf_ctx_sync(ctx.handle))
    for i, x in enumerate(descs):
        ow, ov, (on, os_, of) = O.bow_transform(tree, x, 1)
        a, b = nw[i].item(), nf[i].item()
        assert np.array_equal(w[i, :a].cpu().numpy(), ow) and np.array_equal(v[i, :a].cpu().numpy(), ov)
        assert np.array_equal(nodes[i, :b].cpu().numpy(), on) and np.array_equal(start[i, :b + 1].cpu().numpy(), os_)
        assert np.array_equal(feats[i, :os_[-1]].cpu().numpy(), of)


def _pair(seed, n_a, n_b, noise=8, frac_mp=0.8):
    voc = synth_vocabulary(seed, k=10, L=3)
    rng = np.random.default_rng(seed)
    da = vocab_features(voc, n_a, seed + 1, flip=10)
    m = min(n_a, n_b)
    idx = rng.permutation(n_a)[:m]
    db = np.concatenate([flip_bits(rng, da[idx], noise), vocab_features(voc, n_b - m, seed + 2)])
    ka, kb = np.zeros(n_a, KEYPOINT_DTYPE), np.zeros(n_b, KEYPOINT_DTYPE)
    ka["angle"] = rng.uniform(0, 360, n_a)
    kb["angle"][:m] = (ka["angle"][idx] + rng.normal(25, 10, m)) % 360
    kb["angle"][m:] = rng.uniform(0, 360, n_b - m)
    mpa = np.where(rng.uniform(size=n_a) < frac_mp, np.arange(n_a) + 5000, -1).astype(np.int32)
    mpb = np.where(rng.uniform(size=n_b) < frac_mp, np.arange(n_b) + 9000, -1).astype(np.int32)
    V = ORBVocabulary(voc)
    return voc, V, (da, ka, mpa), (db, kb, mpb)


@pytest.mark.parametrize("mode,check_ori,levelsup", [(0, True, 1), (0, False, 1), (1, True, 1), (1, False, 2),
                                                     (0, True, 4)])
def test_search_by_bow_matches_oracle(mode, check_ori, levelsup):
    voc, V, (da, ka, mpa), (db, kb, mpb) = _pair(40 + mode, 1000, 1100)
    fa = V.transform(da, levelsup)[2]
    fb = V.transform(db, levelsup)[2]
    ng, og = search_by_bow(mode, 0.75, check_ori, (fa, da, ka, mpa), (fb, db, kb, mpb))
    no, oo = O.match_bow(mode, 0.75, check_ori, ((fa.nodes, fa.start, fa.feats), da, ka, mpa),
                         ((fb.nodes, fb.start, fb.feats), db, kb, mpb))
    assert ng == no and np.array_equal(og, oo)
    assert ng > 50


def test_search_by_bow_edge_cases():
    voc, V, (da, ka, mpa), (db, kb, mpb) = _pair(60, 300, 5)
    fa, fb = V.transform(da, 1)[2], V.transform(db, 1)[2]
    for mode in (0, 1):
        ng, og = search_by_bow(mode, 0.6, True, (fa, da, ka, mpa), (fb, db, kb, mpb))
        no, oo = O.match_bow(mode, 0.6, True, ((fa.nodes, fa.start, fa.feats), da, ka, mpa),
                             ((fb.nodes, fb.start, fb.feats), db, kb, mpb))
        assert ng == no and np.array_equal(og, oo)
    empty = FeatureVector(np.zeros(0, np.int32), np.zeros(1, np.int32), np.zeros(0, np.int32))
    ng, og = search_by_bow(0, 0.6, True, (empty, da[:0], ka[:0], mpa[:0]), (fb, db, kb, mpb))
    assert ng == 0 and np.all(og == -1)
