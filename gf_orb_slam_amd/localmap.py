"""Local-map assembly: Tracking::UpdateReference (src/Tracking.cc:3689-3852)
over the C-ABI (gf_update_reference / gf_update_reference_dev,
include/gfslam/abi.h "local-map assembly").

A map is given as flat arrays (`CovisGraph`): keyframes in ascending
KeyFrame* order (the order Map::GetAllKeyFrames and the reference's
std::map<KeyFrame*,int> use) with their isBad flags, map-point slots
(mvpMapPoints) and ordered covisibility lists (mvpOrderedConnectedKeyFrames);
map points with isBad and their observing keyframes (mObservations).
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._lib import check, lib, ptr

_P = ctypes.c_void_p


class CovisMap(ctypes.Structure):
    """gf_covis_map."""

    _fields_ = [("nkf", ctypes.c_int32), ("nmp", ctypes.c_int32), ("kf_bad", _P), ("kf_mp_off", _P), ("kf_mp", _P),
                ("kf_cov_off", _P), ("kf_cov", _P), ("mp_bad", _P), ("mp_obs_off", _P), ("mp_obs", _P)]


_ARRAYS = (("kf_bad", np.uint8), ("kf_mp_off", np.int32), ("kf_mp", np.int32), ("kf_cov_off", np.int32),
           ("kf_cov", np.int32), ("mp_bad", np.uint8), ("mp_obs_off", np.int32), ("mp_obs", np.int32))


class CovisGraph:
    """Host arrays of one map (see module docstring)."""

    def __init__(self, **arrays):
        self.a = {k: np.ascontiguousarray(arrays[k], dt) for k, dt in _ARRAYS}
        self.nkf = len(self.a["kf_bad"])
        self.nmp = len(self.a["mp_bad"])
        assert len(self.a["kf_mp_off"]) == self.nkf + 1 and len(self.a["kf_cov_off"]) == self.nkf + 1
        assert len(self.a["mp_obs_off"]) == self.nmp + 1

    def struct(self) -> CovisMap:
        return CovisMap(self.nkf, self.nmp, *[self.a[k].ctypes.data if self.a[k].size else None for k, _ in _ARRAYS])

    def to_device(self, device="cuda") -> "DeviceCovisGraph":
        return DeviceCovisGraph(self, device)


class DeviceCovisGraph:
    """The same arrays resident on the device (torch allocations as plumbing)."""

    def __init__(self, g: CovisGraph, device="cuda"):
        import torch

        self.nkf, self.nmp = g.nkf, g.nmp
        self.t = {k: torch.from_numpy(np.ascontiguousarray(v) if v.size else np.zeros(1, v.dtype)).to(device)
                  for k, v in g.a.items()}

    def struct(self) -> CovisMap:
        return CovisMap(self.nkf, self.nmp, *[self.t[k].data_ptr() for k, _ in _ARRAYS])


def update_reference(graph: CovisGraph, frame_mps, ctx=None, kf_cap: int | None = None, mp_cap: int | None = None):
    """Tracking::UpdateReference for one frame. Returns (frame_mps with bad
    map points set to -1, local keyframes, local map points, reference
    keyframe index or -1)."""
    from .matcher import default_context

    ctx = ctx or default_context()
    fm = np.array(frame_mps, np.int32, copy=True)
    kf_cap = graph.nkf if kf_cap is None else kf_cap
    mp_cap = graph.nmp if mp_cap is None else mp_cap
    lk = np.zeros(max(kf_cap, 1), np.int32)
    lm = np.zeros(max(mp_cap, 1), np.int32)
    nk, nm, ref = ctypes.c_int(), ctypes.c_int(), ctypes.c_int32()
    m = graph.struct()
    check(lib().gf_update_reference(ctx.handle, ctypes.byref(m), ptr(fm), len(fm), ptr(lk), ctypes.byref(nk),
                                    kf_cap, ptr(lm), ctypes.byref(nm), mp_cap, ctypes.byref(ref)))
    return fm, lk[:nk.value].copy(), lm[:nm.value].copy(), int(ref.value)


def update_reference_batch(dgraph: DeviceCovisGraph, frame_mps, nkps, ctx=None, kf_cap: int | None = None,
                           mp_cap: int | None = None, stream=None):
    """gf_update_reference_dev over B frames (torch int32 tensors on the
    device: frame_mps [B][stride] updated in place, nkps [B]). Returns device
    tensors (local_kfs [B][kf_cap], n_local_kfs [B], local_mps [B][mp_cap],
    n_local_mps [B], ref_kf [B])."""
    import torch

    from .matcher import default_context

    ctx = ctx or default_context()
    B, stride = frame_mps.shape
    kf_cap = dgraph.nkf if kf_cap is None else kf_cap
    mp_cap = dgraph.nmp if mp_cap is None else mp_cap
    dev = frame_mps.device
    lk = torch.zeros((B, max(kf_cap, 1)), dtype=torch.int32, device=dev)
    lm = torch.zeros((B, max(mp_cap, 1)), dtype=torch.int32, device=dev)
    nk = torch.zeros(B, dtype=torch.int32, device=dev)
    nm = torch.zeros(B, dtype=torch.int32, device=dev)
    ref = torch.zeros(B, dtype=torch.int32, device=dev)
    m = dgraph.struct()
    s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
    check(lib().gf_update_reference_dev(ctx.handle, ctypes.byref(m), B, _P(frame_mps.data_ptr()),
                                        _P(nkps.data_ptr()), stride, _P(lk.data_ptr()), _P(nk.data_ptr()), kf_cap,
                                        _P(lm.data_ptr()), _P(nm.data_ptr()), mp_cap, _P(ref.data_ptr()), _P(s)))
    return lk, nk, lm, nm, ref
