"""The batched tracking front end (gf_frontend_*, pipeline.FrontEnd) against
the CPU oracle chain (oracle/chain.cpp) on rendered sequences.

Every step, each checked stream's carried-over state is copied from the
device into the oracle, the oracle tracks the same frame, and every field is
compared: keypoints, descriptors, match indices, scores, outlier flags,
views, updateAtFrameId stamps, leftovers, std::rand() state and the stage
counters bit-exact; poses and the motion model within 1e-5 relative
(north_star); observability blocks within 1e-9 relative (f64 transcendental
ulps in the motion prediction). A second oracle runs the same streams free
(no copy-in) and must stay in agreement with the device frame after frame.
"""
import numpy as np
import pytest

import oracle_chain as C
import oracle_lib as O
from gf_orb_slam_amd import scene, synth
from gf_orb_slam_amd.pipeline import CK, STATS, ck_offsets

EXACT = ["kps", "desc", "nkp", "kp2mp", "score", "outlier", "last_kps", "last_desc", "last_nkp", "last_kp2mp",
         "last_outlier", "last_pos", "views", "mp_upd", "rng", "t_prev", "t_cur"]
POSE = ["Tcw", "velocity", "Tcw_last"]
F64 = ["Xv", "Xv_next", "base", "mp_H", "mp_info", "mp_uv"]
STATE = C.Chain.STATE + ["stats"]


def _setup(camera, nfeat, B, nmap, budget, gf=True, seed=3, n_scenes=2, stale=0.0, dist=None, score_type=1):
    import torch

    from gf_orb_slam_amd.pipeline import FrontEnd

    W = scene.Workload(camera, B, n_scenes=n_scenes, period=32, seed=seed, stale_desc=stale, dist=dist)
    frames = W.render_all("cuda").contiguous()
    maps = W.build_maps(lambda im: O.extract(im, nfeatures=nfeat, score_type=score_type), nmap)
    fe = FrontEnd(camera, nfeat, B, nmap, budget, gf=gf, dist=dist, score_type=score_type)
    for b in range(B):
        fe.set_map(b, *maps[W.scene_of[b]])
        fe.set_rng(b, 1 + seed * 1000 + b)
    fe.set_source(frames, W.scene_of, W.phase)
    T, V = W.boot_state()
    fe.bootstrap(T, V, 0.0)
    torch.cuda.synchronize()
    return W, frames.cpu().numpy(), maps, fe, T, V


def _img(W, frames, b, k):
    return frames[W.scene_of[b], (W.phase[b] + k) % W.period]


def _compare(dev, ch, b, name_prefix=""):
    for k in EXACT:
        a, o = dev[k][b], ch.read(k)
        if k == "left":
            continue
        assert np.array_equal(a, o), f"{name_prefix}{k} differs (stream {b})"
    nl = int(ch.stats()["nleft"])
    assert np.array_equal(dev["left"][b][:nl], ch.read("left")[:nl]), f"{name_prefix}leftovers differ (stream {b})"
    for k in POSE:
        a, o = dev[k][b].astype(np.float64), ch.read(k).astype(np.float64)
        assert np.all(np.abs(a - o) <= 1e-5 * np.maximum(1, np.abs(o))), f"{name_prefix}{k} differs (stream {b})"
    for k in F64:
        np.testing.assert_allclose(dev[k][b], ch.read(k), rtol=1e-9, atol=1e-12,
                                   err_msg=f"{name_prefix}{k} (stream {b})")
    sd = dev["stats"][:, b]
    so = ch.read("stats")
    assert np.array_equal(sd, so), f"{name_prefix}stage counters differ (stream {b}): {sd} vs {so}"


CASES = {
    # config 2 as the bench times it (SURVEY §8d recipe): 93% stale map
    # descriptors, ~60 motion-model matches vs GF budget 100, so
    # runActiveMapMatching runs every frame with ~40 points to match
    "config2_gf": ("euroc", 1000, 4, 2000, 100, True, 0.93),
    # config 2 with every map descriptor current: the matches carried from the
    # last frame exceed the budget (leftovers-only steady state)
    "config2": ("euroc", 1000, 4, 2000, 100, True, 0.0),
    # the same with a GF budget above the tracked count: runActiveMapMatching every frame
    "config2_active": ("euroc", 1000, 4, 2000, 400, True, 0.0),
    # config 3: TUM 640x480, 2000 feats, GF budget 160, 3000-point local map
    "config3": ("tum", 2000, 3, 3000, 160, True, 0.0),
    "config3_gf": ("tum", 2000, 3, 3000, 160, True, 0.93),
    # ORB-SLAM baseline matching (GF off)
    "baseline": ("euroc", 1000, 3, 2000, 100, False, 0.0),
    # distorted cameras (Frame::UndistortKeyPoints, ComputeImageBounds in the
    # step): EuRoC cam0's k1 k2 p1 p2, TUM fr2's five coefficients
    "config2_dist": ("euroc", 1000, 4, 2000, 100, True, 0.93, synth.DISTORTION["euroc"]),
    "config3_dist": ("tum", 2000, 3, 3000, 160, True, 0.0, synth.DISTORTION["tum"]),
    # ORBextractor.nScoreType = HARRIS_SCORE (0) in the settings; 500 features
    "config2_harris": ("euroc", 500, 3, 2000, 100, True, 0.93, None, 0),
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(CASES))
def test_sequence_matches_oracle(case):
    camera, nfeat, B, nmap, budget, gf, stale = CASES[case][:7]
    dist = CASES[case][7] if len(CASES[case]) > 7 else None
    st = CASES[case][8] if len(CASES[case]) > 8 else 1
    W, frames, maps, fe, T, V = _setup(camera, nfeat, B, nmap, budget, gf, stale=stale, dist=dist, score_type=st)
    free = []
    for b in range(B):
        ch = C.Chain(camera, nfeat, nmap, budget, gf, dist=dist, score_type=st)
        ch.set_map(*maps[W.scene_of[b]])
        ch.set_rng(1 + 3 * 1000 + b)
        ch.bootstrap(_img(W, frames, b, 0), T[b], V[b])
        free.append(ch)
    dev = C.read_state(fe)
    for b in range(B):
        for k in ("last_kps", "last_kp2mp", "views", "Tcw_last", "last_pos"):
            assert np.array_equal(dev[k][b], free[b].read(k)), f"bootstrap {k} (stream {b})"
    branches = []
    nsteps = 12
    for k in range(1, nsteps + 1):
        before = dev
        fe.step()
        dev = C.read_state(fe)
        for b in range(B):
            ch = C.Chain(camera, nfeat, nmap, budget, gf, dist=dist, score_type=st)
            ch.load_from(before, b)
            ch.step(_img(W, frames, b, k))
            _compare(dev, ch, b, f"step {k}: ")
            free[b].step(_img(W, frames, b, k))
            _compare(dev, free[b], b, f"free-running step {k}: ")
            branches.append(int(dev["stats"][3, b]))
            assert dev["stats"][14, b] & 4 == 0, "track lost"
    if case == "config2_active":
        assert branches.count(3) >= len(branches) // 4
    if case.endswith("_gf"):
        assert branches.count(3) >= 0.9 * len(branches)  # active matching on (nearly) every frame
    if case == "config2":
        assert branches.count(1) >= len(branches) // 2  # the steady state: matches carried from the last frame
    fe.close()


@pytest.mark.gpu
@pytest.mark.parametrize("stale,budget", [(0.93, 100), (0.0, 100)])
def test_update_reference_in_step(stale, budget):
    """Keyframe graphs (gf_frontend_set_covis): every step runs
    Tracking::UpdateReference on the frame's matches and tracks the rest of
    the frame against that local map (Tracking.cc:2745, 3689-3852). 24
    keyframes of a mapping sweep around the room; the device and the oracle chain (the same
    UpdateReference, gather and scatter) agree on every field for 10 frames,
    free-running and with state copy-in, and the local map changes with the
    frame."""
    import torch

    from gf_orb_slam_amd.pipeline import FrontEnd

    B, G = 3, 2600
    W = scene.Workload("euroc", B, n_scenes=3, period=32, seed=4, stale_desc=stale)
    frames = W.render_all("cuda").contiguous()
    gmaps = W.build_global_maps(lambda im: O.extract(im), G)
    fe = FrontEnd("euroc", 1000, B, G, budget)
    free = []
    T, V = W.boot_state()
    for b in range(B):
        gm = gmaps[W.scene_of[b]]
        fe.set_map(b, gm["mp"], gm["desc"])
        fe.set_covis(b, gm["graph"])
        fe.set_rng(b, 7 + b)
    fe.set_source(frames, W.scene_of, W.phase)
    fe.bootstrap(T, V, 0.0)
    torch.cuda.synchronize()
    fr = frames.cpu().numpy()
    for b in range(B):
        gm = gmaps[W.scene_of[b]]
        ch = C.Chain("euroc", 1000, G, budget)
        ch.set_map(gm["mp"], gm["desc"])
        ch.set_covis(gm["graph"])
        ch.set_rng(7 + b)
        ch.bootstrap(_img(W, fr, b, 0), T[b], V[b])
        free.append(ch)
    dev = C.read_state(fe)
    nlocal = []
    for k in range(1, 11):
        before = dev
        fe.step()
        dev = C.read_state(fe)
        for b in range(B):
            gm = gmaps[W.scene_of[b]]
            ch = C.Chain("euroc", 1000, G, budget)
            ch.load_from(before, b)
            ch.set_covis(gm["graph"])
            ch.step(_img(W, fr, b, k))
            _compare(dev, ch, b, f"refmap step {k}: ")
            free[b].step(_img(W, fr, b, k))
            _compare(dev, free[b], b, f"refmap free-running step {k}: ")
            assert dev["stats"][14, b] & 4 == 0, "track lost"
        nlocal.append(dev["stats"][C.STATS.index("nlocal")].copy())
    nl = np.array(nlocal)
    assert (nl > 0).all() and (nl < G).any() and len(np.unique(nl)) > 1, nl
    fe.close()


FLAG_CAPS = 8 | 16 | 32 | 64 | 128 | 256 | 512 | 1024  # GF_ST_FLAGS bits of the time caps


def _budget_steps(fe, W, frames, B, M, budget, nsteps, set_budgets=None, check=None):
    """Step the device, and for every checked stream replay the step on the
    oracle chain from the state before it, handing the chain only the clock
    record the device wrote (the chain decides every cut itself). Returns the
    per-(step, stream) stats and clock records."""
    dev = C.read_state(fe)
    out = []
    for k in range(1, nsteps + 1):
        if set_budgets:
            set_budgets(k, dev)
        before = dev
        fe.step()
        dev = C.read_state(fe)
        for b in (range(B) if check is None else check):
            ch = C.Chain("euroc", 1000, M, budget)
            ch.load_from(before, b)
            ch.set_clock(dev["clock"][b])
            ch.step(_img(W, frames, b, k))
            _compare(dev, ch, b, f"budgets step {k}: ")
            out.append((dev["stats"][:, b].copy(), dev["clock"][b].copy()))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("match_s,select_s", [(0.0, 0.0), (0.0, 1e9), (1e9, 0.0), (1e9, 1e9), (0.015, 0.098)])
def test_budgets_match_oracle(match_s, select_s):
    """gf_set_budgets: the reference's time caps on the device clock
    (Tracking.cc:866, 3251-3344, 1727-1779, 3097-3137; Observability.cc:
    564-578, 1260-1370; ORBmatcher.cc:276-371). The oracle chain is not told
    where a cut fell: it applies each cap rule to the elapsed times the device
    recorded (GF_FE_CLOCK) and must reach the same state. Budget 0 cuts the
    isInFrustum loop at its first unmatched point (every local point after it
    to mLeftMapPoints) and leaves SearchAdditionalMatchesInFrame no time; the
    reference's own budgets (15 ms match, 98 ms post-publish at 20 fps) cut
    nothing at the device's step times."""
    M = 2000
    W, frames, maps, fe, T, V = _setup("euroc", 1000, 4, M, 100, stale=0.93)
    fe.set_budgets(match_s, select_s)
    res = _budget_steps(fe, W, frames, 4, M, 100, 6)
    fl = np.array([st[STATS.index("flags")] for st, _ in res])
    ntm = np.array([st[STATS.index("to_match")] for st, _ in res])
    extra = np.array([st[STATS.index("extra")] for st, _ in res])
    ncut = np.array([st[STATS.index("ncut")] for st, _ in res])
    if match_s == 0.0:
        assert (fl[ntm > 0] & 32).all() and (ncut[ntm > 0] > 0).all() and not (fl[ntm <= 0] & 32).any()
    if select_s == 0.0:
        assert (fl & 16).all() and (extra == 0).all()
    if match_s >= 1e9:
        assert not (fl & (32 | 64 | 128)).any()
    if select_s >= 1e9:
        assert not (fl & (16 | 256 | 512 | 1024)).any()
    if (match_s, select_s) == (0.015, 0.098):
        assert not (fl & FLAG_CAPS).any(), "the reference's budgets cut a loop at device step times"
    fe.close()


@pytest.mark.gpu
def test_budget_cut_positions_match():
    """A match budget below the isInFrustum loop's time, calibrated on this
    box's clock: the cap fires inside the loop (Tracking.cc:3262-3270), and
    the oracle chain, applying the reference's rule to the device-recorded
    per-point elapsed times, cuts at the same point (stats, leftovers and every
    state field identical). A wide batch spreads the clock reads over many
    waves; 17 streams are replayed."""
    M, B = 2000, 128
    check = list(range(0, B, 8)) + [B - 1]
    W, frames, maps, fe, T, V = _setup("euroc", 1000, B, M, 100, stale=0.93)
    off = ck_offsets(M, 100)

    def calibrate(k, dev):
        if k == 1:  # measure: budgets far above the step record every clock and cut nothing
            fe.set_budgets(1e9, 1e9)
            return
        clk, m = dev["clock"], dev["nmp"]
        el = np.concatenate([clk[b, off["viz"]:off["viz"] + m[b]] for b in range(B)])
        fe.set_budgets(2 * float(np.quantile(el[el >= 0], 0.1 * k)) / 1e8, 1e9)

    res = _budget_steps(fe, W, frames, B, M, 100, 9, calibrate, check)
    fl = np.array([st[STATS.index("flags")] for st, _ in res[len(check):]])
    ncut = np.array([st[STATS.index("ncut")] for st, _ in res[len(check):]])
    mid = int(((ncut > 0) & (ncut < 1900)).sum())
    print("isInFrustum cuts:", int((fl & 32).astype(bool).sum()), "of", len(fl), "frames; mid-list:", mid)
    assert (fl & 32).any(), "no isInFrustum cut at a budget below the loop's time"
    fe.close()


@pytest.mark.gpu
def test_budget_cut_positions_select():
    """timeCost_rest aimed, on this box's clock, at the post-publish caps'
    windows: RunMapPointsSelection's MAP_INFO batches (Tracking.cc:1779 ->
    Observability.cc:573-578) and SearchByProjection_Budget's points
    (ORBmatcher.cc:366-371). A calibration step records where their clock
    reads fall after the timer start; later steps set the budget so the rest
    lands inside one window, up to the step-to-step jitter of timeCost_sofar.
    The oracle chain replays every step from the recorded times."""
    M, B = 2000, 1
    W, frames, maps, fe, T, V = _setup("euroc", 1000, B, M, 100, stale=0.93)
    off = ck_offsets(M, 100)
    win = {}

    def calibrate(k, dev):
        clk = dev["clock"]
        if k == 1:
            fe.set_budgets(1e9, 1e9)
            return
        if k == 2:  # the windows, from the measuring step
            sel = np.concatenate([clk[b, off["sel"]:off["sel"] + (int(dev["nmp"][b]) + 63) // 64] for b in range(B)])
            nl = dev["stats"][STATS.index("nleft")]
            bud = np.concatenate([clk[b, off["bud"]:off["bud"] + nl[b]] for b in range(B)])
            win["map_info"] = float(np.median(sel))
            win["budget"] = float(np.median(clk[:, CK["sa_sofar"]]) + (np.median(bud) if bud.size else 0))
        target = win["map_info"] if k % 2 == 0 else win["budget"]
        fe.set_budgets(1e9, (float(np.median(clk[:, CK["sofar"]])) + target) / 1e8)

    res = _budget_steps(fe, W, frames, B, M, 100, 120, calibrate)
    fl = np.array([st[STATS.index("flags")] for st, _ in res[B:]])
    caps = {bit: int((fl & bit).astype(bool).sum()) for bit in (16, 256, 512, 1024)}
    print("post-publish caps:", caps, "windows (ticks):", win)
    # the windows are a few microseconds wide against tens of jitter, so a
    # few of the 119 steps land in them (8 on the r04 box). Every step's state
    # is checked against the oracle either way (gating); whether a cap fired
    # depends on the box's clock, so it is reported, not asserted
    # (test_budget_cut_positions_exact pins every cap on a test clock)
    if caps[256] + caps[1024] == 0:
        import warnings

        warnings.warn("no wall-clock cap fired inside RunMapPointsSelection or SearchByProjection_Budget")
    fe.close()


def _sec(ticks):  # seconds that gf_set_budgets turns back into exactly `ticks`
    return (ticks + 0.5) / 1e8


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["viz", "active_round", "map_info_select", "budget_matcher"])
def test_budget_cut_positions_exact(case):
    """Each time cap fires at a chosen point, on a test clock
    (gf_frontend_set_test_clock: the check at position idx of a site reads
    base + idx * slope ticks, idx = list point / 64-point batch / round). The
    expected cut follows from the reference's rule alone; the oracle chain,
    replaying the clock record, must reach the same state.
    - viz: isInFrustum, el[i] = 10 i, time_total_match 10000: the loop breaks
      at the first unmatched point with el > 5000, i >= 501 (Tracking.cc
      :3262-3270);
    - active_round: rounds read 100 r, time_for_match = 350 (time_Viz and
      time_Mat_Online 0): round 4 is the first past the cap
      (Observability.cc:1366-1370);
    - map_info_select: timeCost_sofar 1000, select budget 1000 + 750:
      batches read 100 w, batch w is late when 100 w > 750: the first late
      batch is 8 (Tracking.cc:866, 1779; Observability.cc:573-578);
    - budget_matcher: timeCost_rest 50, points read 10 k: the first point that
      reaches the check with 2 * 10 k >= 2 * 50 breaks the loop, k >= 5
      (ORBmatcher.cc:366-371)."""
    M, B = 2000, 4
    W, frames, maps, fe, T, V = _setup("euroc", 1000, B, M, 100, stale=0.93)
    off = ck_offsets(M, 100)
    clock = {"viz": ({"viz": (0, 10)}, 10000, 1e9),
             "active_round": ({"am_round": (0, 100)}, 350, 1e9),
             "map_info_select": ({"sofar": (1000, 0), "sel": (0, 100)}, 1e9, 1750),
             "budget_matcher": ({"sofar": (1000, 0), "bud": (0, 10)}, 1e9, 1050)}[case]
    sites, mt, stt = clock
    fe.set_test_clock(sites)
    fe.set_budgets(_sec(mt) if mt < 1e9 else 1e9, _sec(stt) if stt < 1e9 else 1e9)
    res = _budget_steps(fe, W, frames, B, M, 100, 4)
    fired = 0
    for st, rec in res:
        fl = int(st[STATS.index("flags")])
        if case == "viz":
            n = int(rec[CK["viz_cut"]])
            if st[STATS.index("to_match")] > 0:
                assert np.array_equal(rec[off["viz"]:off["viz"] + 600], 10 * np.arange(600))
                assert fl & 32 and 501 <= n < 501 + 100, (fl, n)
                fired += 1
        elif case == "active_round":
            if rec[CK["am_cut"]] >= 0:
                assert np.array_equal(rec[off["am"]:off["am"] + 5], 100 * np.arange(5))
                assert fl & 128 and rec[CK["am_cut"]] == 4, (fl, rec[CK["am_cut"]])
                fired += 1
        elif case == "map_info_select":
            assert rec[CK["sofar"]] == 1000
            assert fl & 256, fl
            assert np.array_equal(rec[off["sel"]:off["sel"] + 8], 100 * np.arange(8))
            fired += 1
        else:
            nl = int(st[STATS.index("nleft")])
            if nl > 5 and rec[CK["budget_cut"]] >= 0:
                assert fl & 1024 and rec[CK["budget_cut"]] >= 5, (fl, rec[CK["budget_cut"]])
                fired += 1
    assert fired >= len(res) // 2, f"cap fired in {fired} of {len(res)} stream-steps"
    fe.set_test_clock(None)
    fe.close()


@pytest.mark.gpu
def test_bench_shape_parity():
    """The timed configuration itself: 1024 streams in 4 groups of 256 (as
    bench.py runs them, each group on its own context / HIP stream, launches
    interleaved, extraction stages chained by gf_frontend_set_gate, keyframe
    maps of 2100 points with UpdateReference every frame), streams {0, 255,
    511} of each group checked for 2 steps."""
    import torch

    from gf_orb_slam_amd.pipeline import FrontEnd, chain_extraction

    G, Bg, M = 4, 256, 2100
    W = scene.Workload("euroc", G * Bg, n_scenes=8, period=32, seed=5, stale_desc=0.82)
    frames = W.render_all("cuda").contiguous()
    gmaps = W.build_global_maps(lambda im: O.extract(im), M)
    T, V = W.boot_state()
    fes = []
    for g in range(G):
        sl = slice(g * Bg, (g + 1) * Bg)
        fe = FrontEnd("euroc", 1000, Bg, M, 100)
        for b in range(Bg):
            gm = gmaps[W.scene_of[g * Bg + b]]
            fe.set_map(b, gm["mp"], gm["desc"])
            fe.set_covis(b, gm["graph"])
            fe.set_rng(b, 1 + g * Bg + b)
        fe.set_source(frames, W.scene_of[sl], W.phase[sl])
        fe.bootstrap(T[sl], V[sl], 0.0)
        fes.append(fe)
    gates = chain_extraction(fes)
    assert len(gates) == G
    torch.cuda.synchronize()
    fr = frames.cpu().numpy()
    check = [0, Bg // 2 - 1, Bg - 1]
    states = [C.read_state(fe, STATE) for fe in fes]
    for k in (1, 2):
        for fe in fes:
            fe.step()
        for g, fe in enumerate(fes):
            dev = C.read_state(fe)
            for b in check:
                ch = C.Chain("euroc", 1000, M, 100)
                ch.load_from(states[g], b)
                ch.set_covis(gmaps[W.scene_of[g * Bg + b]]["graph"])
                ch.step(_img(W, fr, g * Bg + b, k))
                _compare(dev, ch, b, f"group {g} step {k}: ")
            if k == 2:  # the timed regime: active matching on most streams
                assert (dev["stats"][3] == 3).mean() >= 0.8
                nl = dev["stats"][C.STATS.index("nlocal")]
                assert (nl > 1500).all() and (nl <= M).all() and len(np.unique(nl)) > 1, nl
            states[g] = dev
    for fe in fes:
        fe.close()


@pytest.mark.gpu
def test_graph_replay_equals_eager_with_update_reference():
    """A captured step with keyframe graphs (UpdateReference, local-map
    gather / scatter inside the graph) replays to the eager state."""
    import torch

    from gf_orb_slam_amd.pipeline import FrontEnd

    B, M = 3, 2100
    W = scene.Workload("euroc", B, n_scenes=2, period=32, seed=6, stale_desc=0.82)
    frames = W.render_all("cuda").contiguous()
    gmaps = W.build_global_maps(lambda im: O.extract(im), M)
    T, V = W.boot_state()
    fes = []
    for _ in range(2):
        fe = FrontEnd("euroc", 1000, B, M, 100)
        for b in range(B):
            gm = gmaps[W.scene_of[b]]
            fe.set_map(b, gm["mp"], gm["desc"])
            fe.set_covis(b, gm["graph"])
            fe.set_rng(b, 11 + b)
        fe.set_source(frames, W.scene_of, W.phase)
        fe.bootstrap(T, V, 0.0)
        fes.append(fe)
    fe, fe2 = fes
    fe2.step()
    fe2.capture_graph()
    fe.step()
    for _ in range(4):
        fe.step()
        fe2.step()
    torch.cuda.synchronize()
    a, b = C.read_state(fe), C.read_state(fe2)
    for k in ("kp2mp", "Tcw", "mp_info", "rng", "views", "stats", "map"):
        assert np.array_equal(a[k], b[k]), k
    for f in fes:
        f.close()


@pytest.mark.gpu
def test_track_priority_stream_equals_default():
    """gf_frontend_set_track_priority: tracking forked onto a high-priority
    stream and joined back gives the same state as one stream, gated as the
    bench runs it."""
    from gf_orb_slam_amd.pipeline import chain_extraction

    runs = []
    for prio in (False, True):
        fes = [_setup("euroc", 1000, 4, 2000, 100, stale=0.93, seed=8)[3] for _ in range(2)]
        chain_extraction(fes)
        if prio:
            for fe in fes:
                fe.set_track_priority(-100)
        for _ in range(4):
            for fe in fes:
                fe.step()
        for fe in fes:
            fe.sync()
        runs.append([C.read_state(fe) for fe in fes])
        for fe in fes:
            fe.close()
    for a, b in zip(*runs):
        for k in ("kp2mp", "Tcw", "mp_info", "rng", "views", "stats"):
            assert np.array_equal(a[k], b[k]), k


@pytest.mark.gpu
def test_split_step_and_ring_order_equal_step():
    """gf_frontend_step_extract + gf_frontend_step_track, and GatedRing's
    launch order over gated front ends, give the state plain gated steps
    give; the split calls fail out of order."""
    from gf_orb_slam_amd.pipeline import GatedRing, chain_extraction, step_all

    runs = []
    for mode in ("step", "split", "ring"):
        fes = [_setup("euroc", 1000, 4, 2000, 100, stale=0.93, seed=8)[3] for _ in range(3)]
        chain_extraction(fes)
        ring = GatedRing(fes)
        for _ in range(4):
            if mode == "step":
                for fe in fes:
                    fe.step()
            elif mode == "split":
                step_all(fes)
            else:
                ring.step()
        ring.finish()
        if mode == "split":
            with pytest.raises(RuntimeError):
                fes[0].step_track()  # nothing extracted
            fes[0].step_extract()
            for bad in (fes[0].step_extract, fes[0].step):
                with pytest.raises(RuntimeError):
                    bad()  # the extracted frame is not tracked yet
            fes[0].step_track()
        for fe in fes:
            fe.sync()
        st = [C.read_state(fe) for fe in fes]
        if mode == "split":  # one step more on front end 0: drop it from the comparison
            st[0] = None
        runs.append(st)
        for fe in fes:
            fe.close()
    for mode, run in zip(("split", "ring"), runs[1:]):
        for g, (a, b) in enumerate(zip(runs[0], run)):
            if b is None:
                continue
            for k in ("kp2mp", "Tcw", "mp_info", "rng", "views", "stats"):
                assert np.array_equal(a[k], b[k]), (mode, g, k)


@pytest.mark.gpu
def test_graph_replay_equals_eager():
    """gf_frontend_capture: a replayed step equals an eager one."""
    W, frames, maps, fe, T, V = _setup("euroc", 1000, 4, 2000, 100)
    W2, _, _, fe2, _, _ = _setup("euroc", 1000, 4, 2000, 100)
    fe2.step()
    fe2.capture_graph()  # records the step without running it
    fe.step()
    for _ in range(4):
        fe.step()
        fe2.step()
    a, b = C.read_state(fe), C.read_state(fe2)
    for k in ("kp2mp", "Tcw", "mp_info", "rng", "views", "stats"):
        assert np.array_equal(a[k], b[k]), k
    fe.close()
    fe2.close()


@pytest.mark.gpu
def test_step_host_equals_source():
    """Frames handed over from host memory (PCIe copy in the step) track the same."""
    W, frames, maps, fe, T, V = _setup("euroc", 1000, 2, 2000, 100)
    W2, _, _, fe2, _, _ = _setup("euroc", 1000, 2, 2000, 100)
    for k in range(1, 4):
        fe.step()
        fe2.step_host(np.stack([_img(W, frames, b, k) for b in range(2)]))
    a, b = C.read_state(fe), C.read_state(fe2)
    for k in ("kp2mp", "Tcw", "mp_info", "rng"):
        assert np.array_equal(a[k], b[k]), k
    fe.close()
    fe2.close()


def test_oracle_chain_tracks_sequence():
    """CPU chain on a CPU-rendered loop: tracking holds against ground truth
    (also what bench.py times as cpu_baseline)."""
    W = scene.Workload("euroc", 1, n_scenes=1, period=32, seed=2, tex_size=512)
    fr = W.render_all("cpu").numpy()
    maps = W.build_maps(lambda im: O.extract(im), 2000)
    T, V = W.boot_state()
    ch = C.Chain("euroc", 1000, 2000, 100)
    ch.set_map(*maps[0])
    ch.set_rng(1)
    ch.bootstrap(_img(W, fr, 0, 0), T[0], V[0])
    assert (ch.read("last_kp2mp") >= 0).sum() > 200
    for k in range(1, 6):
        ch.step(_img(W, fr, 0, k))
        st = ch.stats()
        assert st["inl2"] >= 50 and st["flags"] == 0
        err = np.abs(ch.read("Tcw").reshape(4, 4) - W.gt_pose(0, k)).max()
        assert err < 0.02, err


@pytest.mark.gpu
def test_time_log_columns():
    """gf_frontend_set_time_log: Tracking::SaveTimeLog's columns
    (Tracking.h:254-280) for 12 steps of config 2 with active matching on
    every frame: device-clock stage boundaries in order within a step and
    from step to step, durations that add up, the landmark counts taken from
    the step's own statistics, and the reference's text format. The log does
    not change the tracking: the same steps without it give the same state."""
    from gf_orb_slam_amd.pipeline import TIME_LOG_COLUMNS, TL_SITES

    camera, nfeat, B, nmap, budget, gf, stale = CASES["config2_gf"][:7]
    W, frames, maps, fe, T, V = _setup(camera, nfeat, B, nmap, budget, gf, stale=stale)
    W2, _, _, fe2, _, _ = _setup(camera, nfeat, B, nmap, budget, gf, stale=stale)
    fe.set_time_log(16)
    nsteps = 12
    stats = []
    for _ in range(nsteps):
        fe.step()
        fe2.step()
        stats.append(fe.read("stats").copy())
    log = fe.time_log()
    for c in TIME_LOG_COLUMNS:
        assert c in log and log[c].shape == (nsteps, B), c
    st = log["stamps"][:, :len(TL_SITES)]
    assert np.all(st > 0), "every boundary of a GF step is reached"
    assert np.all(np.diff(st, axis=1) >= 0), "boundaries in stage order"
    assert np.all(st[1:, 0] >= st[:-1, -1]), "a step starts after the previous one ended"
    assert np.array_equal(log["recs"]["step"][:, 0], np.arange(log["recs"]["step"][0, 0],
                                                               log["recs"]["step"][0, 0] + nsteps))
    ts = log["frame_time_stamp"]
    assert np.all(np.diff(ts, axis=0) > 0), "frame time stamps increase"
    total = (st[:, -1] - st[:, 0]) * 1e-8
    parts = (log["time_ORB_extraction"] + log["time_track_motion"] + log["time_track_frame"]
             + log["time_track_map"] + log["time_mat_pred"])
    assert np.all(parts <= total[:, None] + 1e-9)
    assert np.all(log["time_match"] + log["time_optim"] <= log["time_track_map"] + 1e-9)
    assert np.all(log["time_ORB_extraction"] > 0) and np.all(log["time_track_map"] > 0)
    idx = {k: i for i, k in enumerate(STATS)}
    for k in range(nsteps):
        s = stats[k]
        assert np.array_equal(log["lmk_num_refInlier"][k], s[idx["inl2"]])
        assert np.array_equal(log["lmk_num_initTrack"][k], s[idx["found"]])
        assert np.array_equal(log["lmk_num_refTrack"][k], s[idx["found"]] + s[idx["local"]])
        assert np.array_equal(log["lmk_num_BA"][k], s[idx["found"]] + s[idx["local"]] + s[idx["extra"]])
        am = s[idx["branch"]] == 3
        assert np.all(log["time_select"][k][am] > 0) and np.all(log["time_select"][k][~am] == 0)
    import os
    import tempfile

    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "time_log.txt")
        fe.save_time_log(fn, 1)
        lines = open(fn).read().splitlines()
    assert lines[0].startswith("#frame_time_stamp time_ORB_extraction") and len(lines) == nsteps + 1
    assert all(len(ln.split()) == len(TIME_LOG_COLUMNS) for ln in lines[1:])
    for k in ("kp2mp", "rng", "Tcw", "stats"):
        assert np.array_equal(fe.read(k), fe2.read(k)), f"{k} differs with the time log on"
    fe.close()
    fe2.close()
