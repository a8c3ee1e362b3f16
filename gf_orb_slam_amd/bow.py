"""Host-side mirror of the DBoW2 ORB vocabulary (ORB_SLAM::ORBVocabulary =
DBoW2::TemplatedVocabulary<FORB::TDescriptor, FORB>, Thirdparty/DBoW2) and of
ORBmatcher::SearchByBoW (src/ORBmatcher.cc:724-853, 1289-1424) over
libgfslam's C-ABI. The tree lives on the device; transform() and the BoW
search run as HIP kernels (csrc/bow.hip)."""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr
from .orb import KEYPOINT_DTYPE, default_context


class VocabArrays(ctypes.Structure):
    _fields_ = [("k", ctypes.c_int32), ("L", ctypes.c_int32), ("scoring", ctypes.c_int32),
                ("weighting", ctypes.c_int32), ("nnodes", ctypes.c_int32), ("parent", ctypes.c_void_p),
                ("desc", ctypes.c_void_p), ("weight", ctypes.c_void_p), ("is_leaf", ctypes.c_void_p)]


class BowSide(ctypes.Structure):
    _fields_ = [("fv_nodes", ctypes.c_void_p), ("fv_start", ctypes.c_void_p), ("fv_feats", ctypes.c_void_p),
                ("nfv", ctypes.c_int32), ("desc", ctypes.c_void_p), ("kps", ctypes.c_void_p),
                ("mp", ctypes.c_void_p), ("n", ctypes.c_int32)]


def read_vocabulary(path: str) -> dict:
    """Parse an ORB vocabulary file (loadFromTextFile for .txt, loadFromBinaryFile
    otherwise) into the tree arrays; host only."""
    hdr = VocabArrays()
    check(lib().gf_vocab_read(path.encode(), ctypes.byref(hdr)))
    n = hdr.nnodes
    out = {"parent": np.zeros(n, np.int32), "desc": np.zeros((n, 32), np.uint8), "weight": np.zeros(n),
           "is_leaf": np.zeros(n, np.uint8)}
    hdr.parent, hdr.desc = out["parent"].ctypes.data, out["desc"].ctypes.data
    hdr.weight, hdr.is_leaf = out["weight"].ctypes.data, out["is_leaf"].ctypes.data
    check(lib().gf_vocab_read(path.encode(), ctypes.byref(hdr)))
    out.update(k=hdr.k, L=hdr.L, scoring=hdr.scoring, weighting=hdr.weighting)
    return out


def save_vocabulary_binary(tree: dict, path: str) -> None:
    """TemplatedVocabulary::saveToBinaryFile (TemplatedVocabulary.h:1516-1536)
    of tree arrays with the root at index 0 (as read_vocabulary returns them)."""
    t = {k: np.ascontiguousarray(tree[k], dt) for k, dt in
         (("parent", np.int32), ("desc", np.uint8), ("weight", np.float64), ("is_leaf", np.uint8))}
    arr = VocabArrays(tree["k"], tree["L"], tree["scoring"], tree["weighting"], len(t["parent"]),
                      *[t[k].ctypes.data for k in ("parent", "desc", "weight", "is_leaf")])
    check(lib().gf_vocab_save_binary(ctypes.byref(arr), path.encode()))


class FeatureVector:
    """DBoW2::FeatureVector as CSR: nodes ascending, feature indices per node."""

    def __init__(self, nodes: np.ndarray, start: np.ndarray, feats: np.ndarray):
        self.nodes, self.start, self.feats = nodes, start, feats

    def items(self):
        return {int(n): self.feats[self.start[i]:self.start[i + 1]].tolist() for i, n in enumerate(self.nodes)}


class ORBVocabulary:
    """TemplatedVocabulary on the device."""

    def __init__(self, tree: dict | None = None, path: str | None = None, ctx=None):
        self.ctx = ctx or default_context()
        self.handle = ctypes.c_void_p()
        if path is not None:
            check(lib().gf_vocab_load(self.ctx.handle, path.encode(), ctypes.byref(self.handle)))
        else:
            self._tree = {k: np.ascontiguousarray(tree[k], dt) for k, dt in
                          (("parent", np.int32), ("desc", np.uint8), ("weight", np.float64), ("is_leaf", np.uint8))}
            arr = VocabArrays(tree["k"], tree["L"], tree["scoring"], tree["weighting"], len(self._tree["parent"]),
                              *[self._tree[k].ctypes.data for k in ("parent", "desc", "weight", "is_leaf")])
            check(lib().gf_vocab_create(self.ctx.handle, ctypes.byref(arr), ctypes.byref(self.handle)))

    @classmethod
    def from_handle(cls, handle, ctx):
        """Wrap a device vocabulary created by the library (gf_dist_bcast_vocab)."""
        v = cls.__new__(cls)
        v.ctx, v.handle = ctx, handle
        return v

    def checksum(self) -> int:
        """Sum over the device node arrays (descriptors, weights, word ids, CSR),
        for comparing copies across ranks."""
        n = self.info()["nnodes"]
        d = np.zeros((n, 32), np.uint8)
        w = np.zeros(n)
        word = np.zeros(n, np.int32)
        cs = np.zeros(n + 1, np.int32)
        check(lib().gf_vocab_download(self.handle, ptr(d), ptr(w), ptr(word), ptr(cs)))
        return int(d.astype(np.int64).sum() * 31 + word.astype(np.int64).sum() * 7 + cs.astype(np.int64).sum()
                   + int(np.round(w.sum() * 1e6)))

    def info(self) -> dict:
        k, L, n, w = ctypes.c_int(), ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        check(lib().gf_vocab_info(self.handle, ctypes.byref(k), ctypes.byref(L), ctypes.byref(n), ctypes.byref(w)))
        return {"k": k.value, "L": L.value, "nnodes": n.value, "nwords": w.value}

    def transform(self, descriptors: np.ndarray, levelsup: int = 4):
        """transform(features, BowVector, FeatureVector, levelsup) ->
        (words, values, FeatureVector); Frame::ComputeBoW uses levelsup 4."""
        d = np.ascontiguousarray(descriptors, np.uint8).reshape(-1, 32)
        n = len(d)
        words, values = np.zeros(max(n, 1), np.int32), np.zeros(max(n, 1))
        nodes, start, feats = np.zeros(max(n, 1), np.int32), np.zeros(n + 1, np.int32), np.zeros(max(n, 1), np.int32)
        nw, nf = ctypes.c_int(), ctypes.c_int()
        check(lib().gf_bow_transform(self.handle, ptr(d) if n else None, n, levelsup, ptr(words), ptr(values),
                                     ctypes.byref(nw), ptr(nodes), ptr(start), ptr(feats), ctypes.byref(nf)))
        nfv = nf.value
        return (words[:nw.value].copy(), values[:nw.value].copy(),
                FeatureVector(nodes[:nfv].copy(), start[:nfv + 1].copy(), feats[:start[nfv]].copy()))

    def close(self) -> None:
        if self.handle:
            lib().gf_vocab_destroy(self.handle)
            self.handle = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _side(fv: FeatureVector, desc: np.ndarray, kps: np.ndarray, mp: np.ndarray, keep: list):
    a = [np.ascontiguousarray(fv.nodes, np.int32), np.ascontiguousarray(fv.start, np.int32),
         np.ascontiguousarray(fv.feats, np.int32), np.ascontiguousarray(desc, np.uint8),
         np.ascontiguousarray(kps, KEYPOINT_DTYPE), np.ascontiguousarray(mp, np.int32)]
    keep.extend(a)
    p = [x.ctypes.data if x.size else None for x in a]
    return BowSide(p[0], p[1], p[2], len(fv.nodes), p[3], p[4], p[5], len(a[3]))


def search_by_bow(mode: int, nnratio: float, check_ori: bool, a: tuple, b: tuple, ctx=None):
    """ORBmatcher(nnratio, check_ori).SearchByBoW; a, b = (FeatureVector,
    descriptors, keypoints, map point per feature (-1 none)). mode 0 =
    (KeyFrame a, Frame b): returns (n, out[b.n] = a's map point); mode 1 =
    (KeyFrame a, KeyFrame b): (n, out[a.n] = b's map point)."""
    ctx = ctx or default_context()
    keep = []
    sa, sb = _side(*a, keep), _side(*b, keep)
    out = np.full(max(sb.n if mode == 0 else sa.n, 1), -1, np.int32)
    nm = ctypes.c_int()
    check(lib().gf_match_bow(ctx.handle, mode, ctypes.c_float(nnratio), int(check_ori), ctypes.byref(sa),
                             ctypes.byref(sb), ptr(out), ctypes.byref(nm)))
    return nm.value, out[:(sb.n if mode == 0 else sa.n)].copy()
