"""Batched tracking front end: the mirror of Tracking::GrabImage for B
independent sequences, over libgfslam's gf_frontend_* (include/gfslam/abi.h).

One `step()` tracks one frame of every stream entirely on the device
(Tracking.cc:461-917, WORKING state): ORB extraction, TrackWithMotionModel
(SearchByProjection(Cur, Last, 15) + PoseOptimization), TrackLocalMap with
the good-feature SearchReferencePointsInFrustum (updatePWLSVec,
FRAME_INFO_MATRIX, then the leftovers-only / SearchByProjection /
runActiveMapMatching branch) + PoseOptimization, the motion-model update,
the next-frame MAP_INFO_MATRIX prediction, SearchAdditionalMatchesInFrame
and the hand-over to mLastFrame. The state of every stream (last frame, pose,
velocity, map-resident observability blocks, std::rand() state) carries over
from step to step, so a stream is a tracked sequence.

PyTorch is not used here: the library owns its buffers and its stream. The
frames come from device memory (`set_source`, e.g. a rendered sequence in a
torch tensor) or from host memory (`step_host`, PCIe copy included).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import synth
from ._lib import check, lib, ptr
from .matcher import MAP_POINT_DTYPE, MP_VIEW_DTYPE
from .observability import Rng
from .orb import KEYPOINT_DTYPE, Context

RELOC_KF_DTYPE = np.dtype([("query", "<u4"), ("words", "<i4"), ("score", "<f4")])  # gf_reloc_kf

# gf_frontend field ids (abi.h GF_FE_*): name -> (id, dtype, per-stream shape
# with "cap" = keypoint capacity and "M" = map capacity)
FIELDS = {
    "kps": (0, KEYPOINT_DTYPE, ("cap",)),
    "desc": (1, np.uint8, ("cap", 32)),
    "nkp": (2, np.int32, ()),
    "Tcw": (3, np.float32, (16,)),
    "kp2mp": (4, np.int32, ("cap",)),
    "score": (5, np.int32, ("cap",)),
    "outlier": (6, np.uint8, ("cap",)),
    "last_kps": (7, KEYPOINT_DTYPE, ("cap",)),
    "last_desc": (8, np.uint8, ("cap", 32)),
    "last_nkp": (9, np.int32, ()),
    "last_kp2mp": (10, np.int32, ("cap",)),
    "last_outlier": (11, np.uint8, ("cap",)),
    "last_pos": (12, np.float32, ("cap", 3)),
    "Tcw_last": (13, np.float32, (16,)),
    "velocity": (14, np.float32, (16,)),
    "t_prev": (15, np.float64, ()),
    "t_cur": (16, np.float64, ()),
    "map": (17, MAP_POINT_DTYPE, ("M",)),
    "map_desc": (18, np.uint8, ("M", 32)),
    "nmp": (19, np.int32, ()),
    "views": (20, MP_VIEW_DTYPE, ("M",)),
    "Xv": (21, np.float64, (13,)),
    "Xv_next": (22, np.float64, (13,)),
    "base": (23, np.float64, (49,)),
    "mp_H": (24, np.float64, ("M", 14)),
    "mp_info": (25, np.float64, ("M", 49)),
    "mp_uv": (26, np.float32, ("M", 2)),
    "mp_upd": (27, np.int32, ("M",)),
    "rng": (28, np.uint8, (ctypes.sizeof(Rng),)),
    "left": (29, np.int32, ("M",)),
    "stats": (30, np.int32, None),  # [NSTAT][B]
    "hist": (31, np.int32, (8,)),  # running counters: steps per branch [0..4], steps cut by a time cap [5],
                                   # log-dets [6], local matches [7]
    "clock": (32, np.int64, ("CK",)),  # budget clock record of the last step (abi.h GF_CK_*)
    "track": (33, np.int32, (8,)),  # tracking state (abi.h GF_TR_*)
    "reloc": (34, RELOC_KF_DTYPE, (64,)),  # keyframes' relocalisation-query state (gf_reloc_kf)
}
STATS = ["m3", "found", "to_match", "branch", "in_view", "local", "inl1", "inl2", "extra", "nleft", "iter1",
         "iter2", "edges1", "edges2", "flags", "frames", "ldets", "nlocal", "ncut", "cand_last", "cand_proj",
         "tpf", "ncand", "reloc", "ransac"]
# GF_FE_TRACK columns and path codes
TR = {"state": 0, "vel": 1, "since": 2, "path": 3, "query": 4, "ok": 5}
PATHS = {0: "motion model", 1: "previous frame after the motion model", 2: "previous frame", 3: "relocalisation"}

NSTAT = len(STATS)

# per-frame stage log (abi.h GF_TL_*, gf_time_rec): device-clock boundaries of a step
TL_SITES = ["begin", "extracted", "motion", "init_pose", "ref_updated", "frustum", "mat_online", "selected",
            "searched", "optimised", "end"]
TL_NSITE = 12
TIME_REC_DTYPE = np.dtype([("frame_time_stamp", np.float64), ("path", np.int32), ("branch", np.int32),
                           ("found", np.int32), ("tpf", np.int32), ("local", np.int32), ("inliers", np.int32),
                           ("extra", np.int32), ("track_map", np.int32), ("flags", np.int32), ("step", np.int32)])
# Tracking::SaveTimeLog's columns (Tracking.h:254-280), in its order
TIME_LOG_COLUMNS = ["frame_time_stamp", "time_ORB_extraction", "time_track_motion", "time_track_frame",
                    "time_track_map", "time_match", "time_select", "time_optim", "time_mat_pred", "time_mat_online",
                    "lmk_num_refTrack", "lmk_num_refInlier", "lmk_num_initTrack", "lmk_num_BA"]
TICK_S = 1e-8  # s_memrealtime: 100 MHz


def time_log_columns(stamps: np.ndarray, recs: np.ndarray) -> dict:
    """logCurrentFrame per step and stream from the device log: stamps
    [n][TL_NSITE] ticks, recs [n][B] TIME_REC_DTYPE -> {column: [n][B]}.
    Where the reference's timers sit (Tracking.cc): extraction :528;
    TrackWithMotionModel / TrackPreviousFrame :605-615 (a motion-model
    failure logs both); TrackLocalMap :672 (UpdateReference through the
    statistics); time_match = UpdateReference + SearchReferencePointsInFrustum
    (:2813); time_optim = PoseOptimization + statistics (:2814);
    time_mat_online = MAP_INFO_MATRIX (:3339); time_select =
    runActiveMapMatching (the GF selection; the reference's TrackLocalMap at
    :2745 leaves it 0, its variants at :2219 / :2705 time the selection
    there); time_mat_pred = from the motion update to the end of the step
    (:791, :913: PWLS prediction, RunMapPointsSelection,
    SearchAdditionalMatchesInFrame). Landmark counts: initTrack = the
    initial estimate's nmatches (:1635 / :1378, :1400), refTrack =
    SearchReferencePointsInFrustum's nMatched + nMatchesFound (:3409, :2808),
    refInlier = mnMatchesInliers, BA = refTrack + the additional matches
    (:3143). A boundary a stage did not reach reads 0."""
    st = stamps.astype(np.float64)
    n, B = recs.shape
    T = {k: st[:, i][:, None] * np.ones((1, B)) for i, k in enumerate(TL_SITES)}

    def dur(a, b):
        return np.where((T[a] > 0) & (T[b] > 0), (T[b] - T[a]) * TICK_S, 0.0)

    path, br, tm = recs["path"], recs["branch"], recs["track_map"] != 0
    motion = (path == 0) | (path == 1)
    prev = (path == 1) | (path == 2)
    out = {"frame_time_stamp": recs["frame_time_stamp"].copy(),
           "time_ORB_extraction": dur("begin", "extracted"),
           "time_track_motion": np.where(motion, dur("extracted", "motion"), 0.0),
           "time_track_frame": np.where(prev, dur("motion", "init_pose"), 0.0),
           "time_track_map": np.where(tm, dur("init_pose", "optimised"), 0.0),
           "time_match": np.where(tm, dur("init_pose", "searched"), 0.0),
           "time_select": np.where(tm & (br == 3), dur("mat_online", "selected"), 0.0),
           "time_optim": np.where(tm, dur("searched", "optimised"), 0.0),
           "time_mat_pred": dur("optimised", "end"),
           "time_mat_online": np.where(tm & (br == 3), dur("frustum", "mat_online"), 0.0)}
    ref = np.where(tm, recs["found"] + recs["local"], 0)
    out["lmk_num_refTrack"] = ref
    out["lmk_num_refInlier"] = np.where(tm, recs["inliers"], 0)
    out["lmk_num_initTrack"] = np.where(path == 0, recs["found"], np.where(prev, recs["tpf"], 0))
    out["lmk_num_BA"] = np.where(tm, ref + recs["extra"], 0)
    return out


# GF_FE_CLOCK layout (abi.h GF_CK_*): header words, then per-stage elapsed-time
# arrays; M = map capacity, R = max(gf_budget, 1)
CK = {"flags": 0, "match": 1, "select": 2, "viz_cut": 3, "viz_time": 4, "mat_online": 5, "am_cut": 6, "sofar": 7,
      "sa_cut": 8, "sa_sofar": 9, "budget_cut": 10}
CK_HEADER = 16
# test-clock sites (abi.h GF_CK_SITE_*)
CK_SITES = ["viz", "mi", "am_start", "am_round", "sofar", "sel", "sa", "sa_sofar", "bud"]


def ck_offsets(M: int, R: int) -> dict:
    """Offsets of the clock record's arrays: isInFrustum points, MAP_INFO
    batches (active branch), active-matching rounds, MAP_INFO batches
    (kinematic[1]), visibility-pass points, SearchByProjection_Budget points."""
    return {"viz": CK_HEADER, "mi": CK_HEADER + M, "am": CK_HEADER + M + 64, "sel": CK_HEADER + M + 64 + R,
            "sa": CK_HEADER + M + 128 + R, "bud": CK_HEADER + 2 * M + 128 + R, "words": CK_HEADER + 3 * M + 128 + R}


class FrontendParams(ctypes.Structure):
    """gf_frontend_params."""

    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("fx", ctypes.c_float),
                ("fy", ctypes.c_float), ("cx", ctypes.c_float), ("cy", ctypes.c_float),
                ("nfeatures", ctypes.c_int32), ("scale_factor", ctypes.c_float), ("nlevels", ctypes.c_int32),
                ("fast_th", ctypes.c_int32), ("batch", ctypes.c_int32), ("map_cap", ctypes.c_int32),
                ("gf_budget", ctypes.c_int32), ("gf", ctypes.c_int32), ("dt", ctypes.c_double),
                ("dist", ctypes.c_float * 5), ("max_frames", ctypes.c_int32), ("harris_score", ctypes.c_int32)]

    @classmethod
    def make(cls, camera: str, nfeatures: int, batch: int, map_cap: int, gf_budget: int, gf: bool = True,
             fps: float = 20.0, nlevels: int = 8, scale_factor: float = 1.2, fast_th: int = 20, dist=None,
             score_type: int = 1):
        """dist: Camera.k1 k2 p1 p2 [k3] (None / k1 = 0: keypoints used as extracted);
        score_type: ORBextractor.nScoreType (1 FAST_SCORE, 0 HARRIS_SCORE)."""
        w, h, fx, fy, cx, cy = synth.CAMERAS[camera]
        d = list(dist or ()) + [0.0] * (5 - len(dist or ()))
        # mMaxFrames = 18 * camera_fps / 30 (Tracking.cc:153; int of a double)
        return cls(w, h, fx, fy, cx, cy, nfeatures, scale_factor, nlevels, fast_th, batch, map_cap, gf_budget,
                   1 if gf else 0, 1.0 / fps, (ctypes.c_float * 5)(*d), int(18 * fps / 30),
                   1 if score_type == 0 else 0)


def field_shape(name: str, B: int, cap: int, M: int, R: int = 1):
    fid, dt, shp = FIELDS[name]
    if shp is None:
        return fid, dt, (NSTAT, B)
    dims = {"cap": cap, "M": M, "CK": ck_offsets(M, R)["words"]}
    return fid, dt, (B,) + tuple(dims.get(s, s) for s in shp)


class GateEvent:
    """A hipEvent_t for gf_frontend_set_gate (gf_event_create)."""

    def __init__(self, ctx: Context):
        h = ctypes.c_void_p()
        check(lib().gf_event_create(ctx.handle, ctypes.byref(h)))
        self.handle = h

    def __del__(self):
        try:
            lib().gf_event_destroy(self.handle)
        except Exception:
            pass


def step_all(fes: list) -> None:
    """One step of every front end, from one host thread: every extraction
    is enqueued before any tracking, so a gated front end's extraction is
    never queued behind the host's launches of another's tracking."""
    for fe in fes:
        fe.step_extract()
    for fe in fes:
        fe.step_track()


class GatedRing:
    """Steps gated front ends (chain_extraction) from one host thread in the
    launch order that keeps the gate's hand-over short: front end g's
    extraction is enqueued right after g - 1's, before g - 1's tracking, and
    the last front end's tracking is held until the next step's first
    extraction is enqueued (call finish() before reading results)."""

    def __init__(self, fes: list):
        self.fes = list(fes)
        self._held = None  # the front end whose tracking is not enqueued yet

    def step(self) -> None:
        prev = self._held
        for fe in self.fes:
            if prev is fe:  # one front end: its frame is tracked before the next is extracted
                prev.step_track()
                prev = None
            fe.step_extract()
            if prev is not None:
                prev.step_track()
            prev = fe
        self._held = prev

    def finish(self) -> None:
        if self._held is not None:
            self._held.step_track()
            self._held = None


def chain_extraction(fes: list) -> list:
    """Gate the front ends' extraction stages into a ring: front end g waits
    for g - 1's extraction (g = 0 for the last one's, previous step), so the
    bandwidth-bound stages run one at a time and each front end's tracking
    overlaps the next one's extraction. Returns the events."""
    if len(fes) < 2:
        return []
    evs = [GateEvent(fe.ctx) for fe in fes]
    for g, fe in enumerate(fes):
        fe.set_gate(evs[g - 1], evs[g])
    return evs


class FrontEnd:
    """B independent streams, one frame each per step."""

    def __init__(self, camera: str = "euroc", nfeatures: int = 1000, batch: int = 1, map_size: int = 2000,
                 gf_budget: int = 100, gf: bool = True, fps: float = 20.0, ctx: Context | None = None, dist=None,
                 score_type: int = 1):
        self.params = FrontendParams.make(camera, nfeatures, batch, map_size, gf_budget, gf, fps, dist=dist,
                                          score_type=score_type)
        self.cam = synth.CAMERAS[camera]
        self.B, self.M = batch, map_size
        self.R = max(gf_budget, 1)
        if ctx is None:
            import torch

            ctx = Context(torch.cuda.current_device() if torch.cuda.is_available() else 0)
        self.ctx = ctx
        h = ctypes.c_void_p()
        check(lib().gf_frontend_create(ctx.handle, ctypes.byref(self.params), ctypes.byref(h)))
        self.handle = h
        c = ctypes.c_int()
        check(lib().gf_frontend_capacity(h, ctypes.byref(c)))
        self.cap = c.value
        self._keep = None

    def close(self) -> None:
        if self.handle:
            check(lib().gf_frontend_destroy(self.handle))
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ set-up
    def set_source(self, frames, scene_of: np.ndarray, phase: np.ndarray) -> None:
        """frames: device tensor [S][period][H][W] u8 (kept alive here);
        stream b reads scene scene_of[b] starting at phase[b]."""
        S, period, H, W = frames.shape
        assert (W, H) == tuple(self.cam[:2]) and frames.is_contiguous()
        self._keep = frames
        base = frames.data_ptr()
        fb = H * W
        bases = (ctypes.c_void_p * self.B)(*[base + int(s) * period * fb for s in scene_of])
        ph = np.ascontiguousarray(phase, np.int32)
        check(lib().gf_frontend_set_source(self.handle, bases, ptr(ph), period, fb))

    def set_map(self, stream: int, mps: np.ndarray, desc: np.ndarray) -> None:
        mps = np.ascontiguousarray(mps, MAP_POINT_DTYPE)
        desc = np.ascontiguousarray(desc, np.uint8)
        check(lib().gf_frontend_set_map(self.handle, stream, ptr(mps), ptr(desc), len(mps)))

    def set_covis(self, stream: int, graph) -> None:
        """gf_frontend_set_covis: the keyframe graph of the stream's map
        (localmap.CovisGraph or the dict scene.build_global_map returns)."""
        from .localmap import CovisGraph

        g = graph if isinstance(graph, CovisGraph) else CovisGraph(**graph)
        self._graphs = getattr(self, "_graphs", {})
        self._graphs[stream] = g
        check(lib().gf_frontend_set_covis(self.handle, stream, ctypes.byref(g.struct())))

    def set_rng(self, stream: int, seed: int) -> None:
        check(lib().gf_frontend_set_rng(self.handle, stream, ctypes.c_uint32(seed)))

    def set_vocab(self, vocab) -> None:
        """gf_frontend_set_vocab: Frame::ComputeBoW's vocabulary for
        relocalisation (a bow.ORBVocabulary, kept alive here)."""
        self._vocab = vocab
        check(lib().gf_frontend_set_vocab(self.handle, vocab.handle if vocab is not None else None))

    def set_kfdb(self, stream: int, db) -> None:
        """gf_frontend_set_kfdb: the stream's keyframe database (a
        KeyframeDB over the same keyframes as its graph; None detaches)."""
        self._kfdbs = getattr(self, "_kfdbs", {})
        self._kfdbs[stream] = db
        check(lib().gf_frontend_set_kfdb(self.handle, stream, db.device(self.ctx) if db is not None else None))

    def bootstrap(self, Tcw: np.ndarray, V: np.ndarray, t0: float = 0.0) -> None:
        T = np.ascontiguousarray(Tcw, np.float32).reshape(self.B, 16)
        Vv = np.ascontiguousarray(V, np.float32).reshape(self.B, 16)
        check(lib().gf_frontend_bootstrap(self.handle, ptr(T), ptr(Vv), ctypes.c_double(t0)))

    # ------------------------------------------------------------ steps
    def step(self) -> None:
        check(lib().gf_frontend_step(self.handle))

    def step_extract(self) -> None:
        """gf_frontend_step_extract: the step's extraction gate and Frame
        construction only (step_track completes the step)."""
        check(lib().gf_frontend_step_extract(self.handle))

    def step_track(self) -> None:
        check(lib().gf_frontend_step_track(self.handle))

    def step_host(self, imgs: np.ndarray) -> None:
        imgs = np.ascontiguousarray(imgs, np.uint8)
        assert imgs.shape == (self.B, self.cam[1], self.cam[0])
        check(lib().gf_frontend_step_host(self.handle, ptr(imgs)))
        self._host_keep = imgs

    def capture_graph(self) -> None:
        check(lib().gf_frontend_capture(self.handle))

    def set_gate(self, wait_event, done_event) -> None:
        """gf_frontend_set_gate: wait for `wait_event` before extraction,
        record `done_event` after it (GateEvent or None)."""
        self._gate = (wait_event, done_event)  # keep the events alive
        check(lib().gf_frontend_set_gate(self.handle, wait_event.handle if wait_event else None,
                                         done_event.handle if done_event else None))

    def set_gate_stage(self, stage: int) -> None:
        """gf_frontend_set_gate_stage: record the gate's done event after
        extraction stage `stage` (0 resize .. 4 describe, the default)."""
        check(lib().gf_frontend_set_gate_stage(self.handle, int(stage)))

    def set_track_priority(self, priority: int = -1) -> None:
        """gf_frontend_set_track_priority: tracking kernels on a stream of HIP
        priority `priority` (lower = more urgent)."""
        check(lib().gf_frontend_set_track_priority(self.handle, priority))

    def sync(self) -> None:
        check(lib().gf_frontend_sync(self.handle))

    def set_budgets(self, match_s: float = float("inf"), select_s: float = float("inf")) -> None:
        check(lib().gf_set_budgets(self.ctx.handle, ctypes.c_double(match_s), ctypes.c_double(select_s)))

    def set_test_clock(self, sites: dict | None) -> None:
        """gf_frontend_set_test_clock (test-only): each budget check at site s
        reads base + idx * slope ticks, sites = {name: (base, slope)} over
        CK_SITES (absent sites read (0, 0)); None restores the device clock."""
        if sites is None:
            check(lib().gf_frontend_set_test_clock(self.handle, None))
            return
        bad = set(sites) - set(CK_SITES)
        if bad:
            raise ValueError(f"unknown clock sites {sorted(bad)}")
        a = np.zeros((len(CK_SITES), 2), np.int64)
        for name, (base, slope) in sites.items():
            a[CK_SITES.index(name)] = (base, slope)
        check(lib().gf_frontend_set_test_clock(self.handle, ptr(a)))

    def set_time_log(self, steps: int) -> None:
        """gf_frontend_set_time_log: keep the last `steps` steps' stage log (0: off)."""
        check(lib().gf_frontend_set_time_log(self.handle, int(steps)))

    def time_log(self) -> dict:
        """The logged steps, oldest first: {"stamps": [n][TL_NSITE] ticks,
        "recs": [n][B] TIME_REC_DTYPE, column: [n][B] for TIME_LOG_COLUMNS}."""
        cap = 4096
        st = np.zeros((cap, TL_NSITE), np.int64)
        rc = np.zeros((cap, self.B), TIME_REC_DTYPE)
        n = ctypes.c_int()
        check(lib().gf_frontend_read_time_log(self.handle, ptr(st), ptr(rc), ctypes.byref(n)))
        st, rc = st[:n.value], rc[:n.value]
        return {"stamps": st, "recs": rc, **time_log_columns(st, rc)}

    def save_time_log(self, filename: str, stream: int = 0) -> None:
        """Tracking::SaveTimeLog's file for one stream (Tracking.h:251-277)."""
        log = self.time_log()
        with open(filename, "w") as fh:
            fh.write("#frame_time_stamp time_ORB_extraction time_track_motion time_track_frame time_track_map "
                     "time_match ...\n")
            for k in range(len(log["recs"])):
                f = [f"{log[c][k, stream]:.6f}" for c in TIME_LOG_COLUMNS[:10]]
                f += [f"{int(log[c][k, stream]):d}" for c in TIME_LOG_COLUMNS[10:]]
                fh.write(" ".join(f) + "\n")

    # ------------------------------------------------------------ state
    def read(self, name: str) -> np.ndarray:
        fid, dt, shape = field_shape(name, self.B, self.cap, self.M, self.R)
        out = np.zeros(shape, dt)
        check(lib().gf_frontend_read(self.handle, fid, ptr(out), out.nbytes))
        return out

    def write(self, name: str, arr: np.ndarray) -> None:
        fid, dt, shape = field_shape(name, self.B, self.cap, self.M, self.R)
        a = np.ascontiguousarray(arr, dt).reshape(shape)
        check(lib().gf_frontend_write(self.handle, fid, ptr(a), a.nbytes))

    def stats(self) -> dict:
        s = self.read("stats")
        return {k: s[i] for i, k in enumerate(STATS)}

    # ------------------------------------------------------------ profiling
    def prof_enable(self, on: bool = True) -> None:
        check(lib().gf_prof_enable(self.ctx.handle, int(on)))

    def prof_reset(self) -> None:
        check(lib().gf_prof_reset(self.ctx.handle))

    def prof_report(self) -> dict:
        out = {}
        i = 0
        name = ctypes.create_string_buffer(64)
        while True:
            ms, cnt = ctypes.c_double(), ctypes.c_int()
            rc = lib().gf_prof_report(self.ctx.handle, i, name, 64, ctypes.byref(ms), ctypes.byref(cnt))
            if rc != 0:
                break
            out[name.value.decode()] = (ms.value, cnt.value)
            i += 1
        return out


def make_workload_frontend(camera: str, nfeatures: int, batch: int, map_size: int, gf_budget: int, workload,
                           frames, maps, seed: int = 0, ctx: Context | None = None) -> FrontEnd:
    """A FrontEnd over a scene.Workload: per-stream maps (of its scene),
    std::srand(1 + seed * 1000 + b), the source frames and the bootstrap at
    the ground-truth pose."""
    fe = FrontEnd(camera, nfeatures, batch, map_size, gf_budget, ctx=ctx)
    for b in range(batch):
        mp, d = maps[workload.scene_of[b]]
        fe.set_map(b, mp, d)
        fe.set_rng(b, 1 + seed * 1000 + b)
    fe.set_source(frames, workload.scene_of, workload.phase)
    T, V = workload.boot_state()
    fe.bootstrap(T, V, 0.0)
    return fe


class KeyframeDBArrays(ctypes.Structure):
    """gf_keyframe_db."""

    _fields_ = [("nkf", ctypes.c_int32)] + [(k, ctypes.c_void_p) for k in
                                           ("kp_off", "kps", "desc", "bow_off", "bow_words", "bow_values", "fv_off",
                                            "fv_nodes", "fv_start", "fv_feats")]


class KeyframeDB:
    """The keyframes of a map as Relocalisation reads them (abi.h
    gf_keyframe_db): per keyframe its keypoints, descriptors, BowVector and
    FeatureVector (KeyFrame::ComputeBoW, levelsup 4). `transform(desc)` gives
    (words, values, FeatureVector) — the library's ORBVocabulary.transform on
    the device, or a CPU restatement in the oracle tests."""

    def __init__(self, kf_kps: list, kf_desc: list, transform):
        from .orb import KEYPOINT_DTYPE

        self.nkf = len(kf_kps)
        kps = [np.ascontiguousarray(k, KEYPOINT_DTYPE) for k in kf_kps]
        desc = [np.ascontiguousarray(d, np.uint8).reshape(-1, 32) for d in kf_desc]
        self.kp_off = np.zeros(self.nkf + 1, np.int32)
        self.kp_off[1:] = np.cumsum([len(k) for k in kps])
        self.kps = np.concatenate(kps) if kps else np.zeros(0, KEYPOINT_DTYPE)
        self.desc = np.ascontiguousarray(np.concatenate(desc) if desc else np.zeros((0, 32), np.uint8))
        bw, bv, fn, fs, ff = [], [], [], [0], []
        self.bow_off = np.zeros(self.nkf + 1, np.int32)
        self.fv_off = np.zeros(self.nkf + 1, np.int32)
        for k, d in enumerate(desc):
            w, v, fv = transform(d)
            bw.append(np.asarray(w, np.int32))
            bv.append(np.asarray(v, np.float64))
            self.bow_off[k + 1] = self.bow_off[k] + len(w)
            fn.append(np.asarray(fv.nodes, np.int32))
            base = fs[-1]
            fs.extend((base + np.asarray(fv.start[1:], np.int64)).tolist())
            ff.append(np.asarray(fv.feats, np.int32))
            self.fv_off[k + 1] = self.fv_off[k] + len(fv.nodes)
        cat = lambda xs, dt: np.ascontiguousarray(np.concatenate(xs) if xs else np.zeros(0, dt), dt)
        self.bow_words, self.bow_values = cat(bw, np.int32), cat(bv, np.float64)
        self.fv_nodes, self.fv_feats = cat(fn, np.int32), cat(ff, np.int32)
        self.fv_start = np.ascontiguousarray(fs, np.int32)
        self._dev = {}

    def struct(self) -> KeyframeDBArrays:
        a = [self.kp_off, self.kps, self.desc, self.bow_off, self.bow_words, self.bow_values, self.fv_off,
             self.fv_nodes, self.fv_start, self.fv_feats]
        return KeyframeDBArrays(self.nkf, *[x.ctypes.data if x.size else None for x in a])

    def device(self, ctx):
        """The gf_kfdb handle on ctx (created once, shared by the streams)."""
        key = id(ctx)
        if key not in self._dev:
            h = ctypes.c_void_p()
            check(lib().gf_kfdb_create(ctx.handle, ctypes.byref(self.struct()), ctypes.byref(h)))
            self._dev[key] = (ctx, h)  # the context outlives the handle
        return self._dev[key][1]

    def __del__(self):
        try:
            for _, h in self._dev.values():
                lib().gf_kfdb_destroy(h)
        except Exception:
            pass
