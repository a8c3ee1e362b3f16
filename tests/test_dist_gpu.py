"""gf_dist_* (the config-5 start-up exchange inside libgfslam) on the GPU box.

- A single-rank RCCL communicator: the broadcast / all-reduce entry points
  run through RCCL, the vocabulary and map broadcasts keep the root's state
  intact, and bench.py's start-up protocol (GfDist + share_world) returns the
  world it packed.
- The receiving side on one GPU: two and three ranks as threads
  of this process over the loopback transport (gf_dist_init_loopback: a
  rendezvous and device-to-device copies behind the same entry points). Every
  non-root line runs: gf_dist_bcast_vocab's header decode and allocations
  (bow.hip), gf_dist_bcast_map's reset of the receivers' map state
  (frontend.hip), the all-reduces of the checksums. The receivers' vocabulary
  transform and their front ends' first steps (with a relocalisation that
  uses the received vocabulary) then equal the root's, bit for bit.
- Two processes sharing the GPU over the host-staged transport
  (gf_dist_init_host with gloo collectives): the same protocol across a
  process boundary.
The RCCL path at world > 1 needs one GPU per rank (the driver's 8-GPU run)."""
import os
import socket
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_single_rank_rccl_exchange():
    import torch

    from gf_orb_slam_amd import synth
    from gf_orb_slam_amd.bow import ORBVocabulary
    from gf_orb_slam_amd.dist import GfDist, checksum, pack_world, share_world
    from gf_orb_slam_amd.orb import Context
    from gf_orb_slam_amd.pipeline import FrontEnd

    from test_dist_cpu import _build

    ctx = Context(0)
    gd = GfDist(ctx, 0, 1)
    assert gd.transport_kind() == 0
    a = np.arange(1000, dtype=np.uint8)
    assert np.array_equal(gd.bcast_array(a), a)
    span = gd.gather_ints([3.0, 7.0])
    assert np.array_equal(span, [[3.0, 7.0], [3.0, 7.0]])
    scenes, maps, ck, span, nbytes = share_world(gd, 0, _build)
    assert ck == checksum(pack_world(*_build())) and span[0][0] == span[1][0]
    voc = ORBVocabulary(synth.synth_vocabulary(7, k=10, L=3), ctx=ctx)
    c0 = voc.checksum()
    assert gd.bcast_vocab(voc, 0).checksum() == c0
    fe = FrontEnd("euroc", 1000, 2, 100, 100, ctx=Context(0))
    for b in range(2):
        fe.set_map(b, *maps[b])
    before = fe.read("map").copy()
    gd.bcast_map(fe, 0)
    assert np.array_equal(fe.read("map"), before)
    torch.cuda.synchronize()
    fe.close()
    gd.close()


# ------------------------------------------------------------ loopback ranks
B, G, NKF = 4, 2600, 12


def _world_build():
    """Rank 0's world as bench.build_world makes it: two scenes, keyframe
    maps extracted with the product extractor (graph + keyframe keypoints and
    descriptors for the relocalisation databases)."""
    from gf_orb_slam_amd import ORBextractor, scene

    W0 = scene.Workload("euroc", B, n_scenes=2, period=32, seed=3, stale_desc=0.82)
    ex = ORBextractor(1000, 1.2, 8, 1, 20)
    gm = W0.build_global_maps(lambda im: ex(im), G, n_kf=NKF, device="cuda:0")
    return W0.scenes, [(g["mp"], g["desc"], g["graph"], g["kf_kps"], g["kf_desc"]) for g in gm]


def _loopback_rank(rank, world, ch, out, errs):
    """One rank's start-up exchange, as bench.py main() runs it."""
    try:
        import torch

        from gf_orb_slam_amd import scene, synth
        from gf_orb_slam_amd.bow import ORBVocabulary
        from gf_orb_slam_amd.dist import GfDist, checksum, share_world
        from gf_orb_slam_amd.orb import Context
        from gf_orb_slam_amd.pipeline import FrontEnd

        torch.cuda.set_device(0)
        ctx = Context(0)
        gd = GfDist(ctx, rank, world, transport="loopback", channel=ch)
        assert gd.transport_kind() == 1
        scenes, maps, ck, span, nbytes = share_world(gd, rank, _world_build)
        voc = ORBVocabulary(synth.synth_vocabulary_fast(seed=7, k=10, L=5), ctx=ctx) if rank == 0 else None
        voc = gd.bcast_vocab(voc, 0)
        W = scene.Workload("euroc", B, n_scenes=len(scenes), period=32, seed=3, scenes=scenes)
        fe = FrontEnd("euroc", 1000, B, G, 100, ctx=Context(0))
        if rank == 0:
            for b in range(B):
                fe.set_map(b, *maps[W.scene_of[b]][:2])
        gd.bcast_map(fe, 0)
        vspan = gd.gather_ints([voc.checksum(), checksum(fe.read("map")), checksum(fe.read("map_desc"))])
        out[rank] = dict(gd=gd, ctx=ctx, scenes=scenes, maps=maps, ck=ck, span=span, voc=voc, W=W, fe=fe,
                         vspan=vspan)
    except Exception as e:  # noqa: BLE001 - reported by the test body
        import traceback

        errs.append((rank, repr(e), traceback.format_exc()))


def _run_loopback(world):
    from gf_orb_slam_amd.dist import LoopbackChannel

    ch = LoopbackChannel(world)
    out, errs = {}, []
    th = [threading.Thread(target=_loopback_rank, args=(r, world, ch, out, errs)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=600)
    assert not any(t.is_alive() for t in th), "a loopback rank did not finish"
    assert not errs, errs
    return ch, out


@pytest.mark.parametrize("world", [2, 3])
def test_loopback_receivers_track_like_the_root(world):
    import torch

    import oracle_chain as C
    from gf_orb_slam_amd.dist import checksum, pack_world
    from gf_orb_slam_amd.pipeline import STATS, TR, KeyframeDB

    ch, out = _run_loopback(world)
    root = out[0]
    for r in range(world):
        o = out[r]
        assert o["ck"] == root["ck"] and np.all(o["span"][0] == o["span"][1])
        assert checksum(pack_world(o["scenes"], o["maps"])) == root["ck"]
        assert np.all(o["vspan"][0] == o["vspan"][1]), o["vspan"]  # vocabulary and map checksums
        assert o["voc"].info() == root["voc"].info()
    # the received vocabulary transforms like the root's (words, weights, FeatureVector)
    rng = np.random.default_rng(5)
    d = rng.integers(0, 256, (700, 32), dtype=np.uint8)
    w0, v0, f0 = root["voc"].transform(d)
    for r in range(1, world):
        w, v, f = out[r]["voc"].transform(d)
        assert np.array_equal(w, w0) and np.array_equal(v, v0)
        assert np.array_equal(f.nodes, f0.nodes) and np.array_equal(f.start, f0.start) and \
            np.array_equal(f.feats, f0.feats)
    # every rank tracks the same sequences (same phases here): a blank pair of
    # frames sends stream 0 LOST, its relocalisation runs on each rank's own
    # (received) vocabulary and keyframe database
    for r in range(world):
        o = out[r]
        W, fe = o["W"], o["fe"]
        fr = W.render_all("cuda:0").contiguous()
        s0 = W.scene_of[0]
        for k in (2, 3):
            fr[s0, (W.phase[0] + k) % W.period] = 100
        o["frames"] = fr
        dbs = [KeyframeDB(m[3], m[4], o["voc"].transform) for m in o["maps"]]
        fe.set_vocab(o["voc"])
        for b in range(B):
            fe.set_covis(b, o["maps"][W.scene_of[b]][2])
            fe.set_kfdb(b, dbs[W.scene_of[b]])
            fe.set_rng(b, 11 + b)
        fe.set_source(fr, W.scene_of, W.phase)
        T, V = W.boot_state()
        fe.bootstrap(T, V, 0.0)
        o["dbs"] = dbs
    torch.cuda.synchronize()
    names = [k for k in C.FIELDS if k != "clock"]
    paths = []
    for step in range(1, 7):
        states = []
        for r in range(world):
            out[r]["fe"].step()
            out[r]["fe"].sync()
            states.append(C.read_state(out[r]["fe"], names))
        for r in range(1, world):
            for k in names:
                assert np.array_equal(states[r][k], states[0][k]), f"step {step}: rank {r} field {k} differs"
        st = states[0]["stats"]
        paths.append(int(states[0]["track"][0][TR["path"]]))
        assert st[STATS.index("frames"), 0] >= step
    assert 3 in paths, f"stream 0 never relocalised: {paths}"
    for r in range(world):
        out[r]["fe"].close()
        out[r]["gd"].close()
    ch.close()


# ------------------------------------------------- host-staged, two processes
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _host_rank(rank, world, port, q):
    try:
        import torch
        import torch.distributed as dist

        from gf_orb_slam_amd import synth
        from gf_orb_slam_amd.bow import ORBVocabulary
        from gf_orb_slam_amd.dist import GfDist, checksum, share_world
        from gf_orb_slam_amd.orb import Context
        from gf_orb_slam_amd.pipeline import FrontEnd

        from test_dist_cpu import _build

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        torch.cuda.set_device(0)
        ctx = Context(0)
        gd = GfDist(ctx, rank, world, transport="host")
        scenes, maps, ck, span, nbytes = share_world(gd, rank, _build)
        voc = ORBVocabulary(synth.synth_vocabulary(7, k=10, L=3), ctx=ctx) if rank == 0 else None
        voc = gd.bcast_vocab(voc, 0)
        fe = FrontEnd("euroc", 1000, 3, 100, 100, ctx=Context(0))
        if rank == 0:
            for b in range(3):
                fe.set_map(b, *maps[b])
        gd.bcast_map(fe, 0)
        rng = np.random.default_rng(9)
        w, v, f = voc.transform(rng.integers(0, 256, (300, 32), dtype=np.uint8))
        res = [voc.checksum(), checksum(fe.read("map")), checksum(fe.read("map_desc")), checksum(fe.read("mp_upd")),
               checksum(w), checksum(v), checksum(f.nodes), checksum(f.feats)]
        span2 = gd.gather_ints(res)
        fe.close()
        gd.close()
        dist.destroy_process_group()
        q.put((rank, ck, bool(np.all(span[0] == span[1])), bool(np.all(span2[0] == span2[1])), None))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, None, False, False, repr(e) + traceback.format_exc()))


def test_host_staged_two_processes_share_one_gpu():
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_host_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=300) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    assert all(r[4] is None for r in res), [r[4] for r in res]
    assert all(p.exitcode == 0 for p in procs)
    assert res[0][1] == res[1][1] and all(r[2] and r[3] for r in res)
