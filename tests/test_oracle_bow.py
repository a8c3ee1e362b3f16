"""Vocabulary loaders (host, no GPU) and the CPU oracle of rows D1 / M6.
DBoW2 is vendored; no DBoW2 test or fixture exists upstream, so the oracle is
pinned by these invariants of the restated text."""
import numpy as np
import pytest

import oracle_lib as O
from gf_orb_slam_amd.bow import read_vocabulary
from gf_orb_slam_amd.synth import synth_vocabulary, vocab_features, write_vocab_binary, write_vocab_text


def test_binary_loader_round_trip_with_duplicate_last_record(tmp_path):
    voc = synth_vocabulary(3, k=5, L=3)
    p = str(tmp_path / "voc.bin")
    write_vocab_binary(voc, p)
    got = read_vocabulary(p)
    n = len(voc["parent"])
    # loadFromBinaryFile reads until eof(): the final failed read re-adds the last record
    assert len(got["parent"]) == n + 1
    for key in ("parent", "desc", "is_leaf"):
        assert np.array_equal(got[key][:n], voc[key])
        assert np.array_equal(got[key][n], voc[key][n - 1])
    assert np.array_equal(got["weight"][:n], voc["weight"].astype(np.float32).astype(np.float64))
    assert (got["k"], got["L"], got["scoring"], got["weighting"]) == (5, 3, 0, 0)


def test_text_loader_round_trip(tmp_path):
    voc = synth_vocabulary(4, k=4, L=2, weighting=1, scoring=1)
    p = str(tmp_path / "voc.txt")
    write_vocab_text(voc, p)
    got = read_vocabulary(p)
    for key in ("parent", "desc", "is_leaf", "weight"):
        assert np.array_equal(got[key], voc[key])
    assert (got["scoring"], got["weighting"]) == (1, 1)


def test_transform_invariants():
    voc = synth_vocabulary(7, k=10, L=3)
    d = vocab_features(voc, 1000, 1)
    words, values, (nodes, start, feats) = O.bow_transform(voc, d, 4)
    assert np.all(np.diff(words) > 0) and np.all(np.diff(nodes) > 0)
    assert abs(values.sum() - 1.0) < 1e-12  # L1 normalised, all weights positive
    assert len(set(feats.tolist())) == len(feats) and np.all(np.diff(start) > 0)
    # levelsup 4 > L: every feature sits at the root node
    assert nodes.tolist() == [0]
    _, _, (nodes2, _, _) = O.bow_transform(voc, d, 1)
    assert len(nodes2) > 10  # level L-1 nodes


def test_duplicate_descriptor_gets_identical_word():
    voc = synth_vocabulary(8, k=6, L=3)
    d = vocab_features(voc, 50, 2)
    w1, v1, _ = O.bow_transform(voc, d)
    w2, v2, _ = O.bow_transform(voc, np.concatenate([d, d]))
    assert np.array_equal(w1, w2) and np.allclose(v1, v2)


def test_match_bow_recovers_correspondences():
    voc = synth_vocabulary(9, k=10, L=3)
    rng = np.random.default_rng(0)
    da = vocab_features(voc, 400, 3, flip=10)
    perm = rng.permutation(400)
    from gf_orb_slam_amd.synth import flip_bits
    db = flip_bits(rng, da[perm], 8)
    from gf_orb_slam_amd.orb import KEYPOINT_DTYPE
    ka, kb = np.zeros(400, KEYPOINT_DTYPE), np.zeros(400, KEYPOINT_DTYPE)
    ka["angle"] = rng.uniform(0, 360, 400)
    kb["angle"] = (ka["angle"][perm] + 20) % 360
    _, _, fa = O.bow_transform(voc, da, 1)
    _, _, fb = O.bow_transform(voc, db, 1)
    mp = np.arange(400, dtype=np.int32) + 1000
    n, out = O.match_bow(0, 0.75, True, (fa, da, ka, mp), (fb, db, kb, np.full(400, -1, np.int32)))
    ok = out >= 0
    assert n == ok.sum() and n > 200
    assert np.all(out[ok] == mp[perm[ok]])  # every accepted match is the true one


def test_bin_vocabulary_tool_matches_save_to_binary(tmp_path):
    """tools/bin_vocabulary.cc: loadFromTextFile + saveToBinaryFile. The
    converter's bytes equal the saveToBinaryFile layout written from the same
    tree, and loading them back gives the text tree plus the binary loader's
    duplicated last record."""
    from gf_orb_slam_amd.bin_vocabulary import convert

    voc = synth_vocabulary(13, k=6, L=3, stop_frac=0.1)
    txt, out, ref = str(tmp_path / "v.txt"), str(tmp_path / "v.bin"), str(tmp_path / "ref.bin")
    write_vocab_text(voc, txt)
    r = convert(txt, out)
    write_vocab_binary(voc, ref)
    assert r["nodes"] == len(voc["parent"])
    assert open(out, "rb").read() == open(ref, "rb").read()
    tb, tt = read_vocabulary(out), read_vocabulary(txt)
    n = len(tt["parent"])
    assert len(tb["parent"]) == n + 1
    for key in ("parent", "desc", "is_leaf"):
        assert np.array_equal(tb[key][:n], tt[key])
    assert np.array_equal(tb["weight"][:n], tt["weight"].astype(np.float32).astype(np.float64))
