"""Host launch orders over gated front ends (pipeline.step_all, GatedRing):
the order of the split-step calls, checked on stand-in front ends (no GPU).
The device state these orders give is checked against plain steps in
test_pipeline_gpu.py::test_split_step_and_ring_order_equal_step."""
from gf_orb_slam_amd.pipeline import GatedRing, step_all


class _FE:
    def __init__(self, g, log):
        self.g, self.log, self.pending = g, log, False

    def step_extract(self):
        assert not self.pending, "extract twice without tracking"
        self.pending = True
        self.log.append(("E", self.g))

    def step_track(self):
        assert self.pending, "track without an extracted frame"
        self.pending = False
        self.log.append(("T", self.g))


def test_step_all_extracts_before_tracking():
    log = []
    fes = [_FE(g, log) for g in range(4)]
    step_all(fes)
    assert log == [("E", 0), ("E", 1), ("E", 2), ("E", 3), ("T", 0), ("T", 1), ("T", 2), ("T", 3)]


def test_gated_ring_order_and_finish():
    log = []
    fes = [_FE(g, log) for g in range(3)]
    ring = GatedRing(fes)
    ring.step()
    # g's extraction is enqueued before g - 1's tracking; the last one's is held
    assert log == [("E", 0), ("E", 1), ("T", 0), ("E", 2), ("T", 1)]
    ring.step()
    assert log[5:] == [("E", 0), ("T", 2), ("E", 1), ("T", 0), ("E", 2), ("T", 1)]
    ring.finish()
    assert log[-1] == ("T", 2) and not any(fe.pending for fe in fes)
    ring.finish()  # idempotent
    assert log[-1] == ("T", 2) and len(log) == 12
    # every front end: extract / track alternate, equal counts
    for g in range(3):
        seq = [k for k, gg in log if gg == g]
        assert seq == ["E", "T"] * 2


def test_gated_ring_single_front_end():
    log = []
    fe = _FE(0, log)
    ring = GatedRing([fe])
    for _ in range(3):
        ring.step()
    ring.finish()
    assert log == [("E", 0), ("T", 0)] * 3
