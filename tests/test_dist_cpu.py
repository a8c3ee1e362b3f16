"""The multi-process path of bench.py on CPU ranks (gloo, world_size 2): the
start-up broadcast reaches every rank and the timed region is the max over
ranks. On the GPU node the same functions run over RCCL."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q):
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    voc, ck = bench.share_startup_state(dist, "cpu", world, rank, vocab_levels=3)
    assert len(voc["parent"]) == 1111 and voc["desc"].shape == (1111, 32)
    t = bench.max_over_ranks(dist, "cpu", world, 1.0 + rank)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, ck, t))


@pytest.mark.parametrize("world", [2])
def test_broadcast_and_max_over_ranks(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cks = {ck for _, ck, _ in res}
    assert len(cks) == 1 and cks.pop() != 0
    assert all(t == float(world) for _, _, t in res)
