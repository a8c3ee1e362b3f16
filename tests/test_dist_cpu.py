"""The config-5 start-up exchange on CPU ranks (gloo, world sizes 2 and 4):
rank 0's world (scenes + local maps) reaches every rank bit-identically
(checksums equal, unpacked arrays equal to rank 0's), every rank then
derives its own sequences (rank-dependent phases), and the timed region is
the max over ranks. On the GPU node the same protocol runs over RCCL
(gf_dist_*, tests/test_dist_gpu.py)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _build():
    from gf_orb_slam_amd import scene
    from gf_orb_slam_amd.matcher import MAP_POINT_DTYPE

    scenes = [scene.Scene(100 + s, tex_size=64) for s in range(3)]
    rng = np.random.default_rng(4)
    maps = []
    for s in range(3):
        mp_ = np.zeros(50 + 10 * s, MAP_POINT_DTYPE)
        mp_["pos"] = rng.uniform(-3, 3, (len(mp_), 3))
        maps.append((mp_, rng.integers(0, 256, (len(mp_), 32), dtype=np.uint8)))
    return scenes, maps


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist

    from gf_orb_slam_amd import scene
    from gf_orb_slam_amd.dist import TorchComm, checksum, pack_world, share_world

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    comm = TorchComm(rank, world)
    scenes, maps, ck, span, nbytes = share_world(comm, rank, _build)
    ref = pack_world(*_build())  # what rank 0 sent
    same = checksum(pack_world(scenes, maps)) == checksum(ref) == ck
    W = scene.Workload("euroc", 12, n_scenes=3, period=32, seed=0, scenes=scenes, phase_offset=3 * rank)
    t = torch.tensor([1.0 + rank], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, ck, bool(np.all(span[0] == span[1])), same, W.phase.tolist(), float(t.item()), nbytes))


@pytest.mark.parametrize("world", [2, 4])
def test_world_broadcast_and_max_over_ranks(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert len({r[1] for r in res}) == 1
    assert all(r[2] and r[3] for r in res)
    assert len({tuple(r[4]) for r in res}) == world  # every rank tracks different sequences
    assert all(r[5] == float(world) for r in res)
    assert all(r[6] > 3 * 7 * 64 * 64 for r in res)


def test_bench_refuses_world_mismatch():
    """bench.py under a launcher whose WORLD_SIZE differs from --gpus exits
    non-zero before touching the GPU."""
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "does not match --gpus" in (r.stderr + r.stdout)
