"""gf_dist_* (RCCL inside libgfslam) on the GPU box with a single-rank
communicator: the broadcast / all-reduce entry points run through RCCL, the
vocabulary and map broadcasts keep the root's state intact, and bench.py's
start-up protocol (GfDist + share_world) returns the world it packed. The
receiving side of the protocol is covered on CPU ranks (test_dist_cpu.py);
more than one rank needs more than one GPU (the driver's 8-GPU run)."""
import numpy as np
import pytest


@pytest.mark.gpu
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
