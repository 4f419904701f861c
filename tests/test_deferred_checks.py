"""The pooling run-count checks a forward defers (PointTransformerV3.check_deferred): a failing
forward raises exactly once, naming its forward id and pooling; its entries leave the pending list before they are
validated, so the model recovers; reads that have not landed stay pending unless the caller waits."""
import pytest

from splatformer_amd.ptv3 import PointTransformerV3


class FakeRead:
    """Stands in for _lib.HostRead: the per-row run ends of one pooling."""

    def __init__(self, ends, ready=True):
        self.ends, self._ready, self.gets = ends, ready, 0

    def get(self):
        self.gets += 1
        return self.ends

    def ready(self):
        return self._ready


def small_model():
    return PointTransformerV3(in_channels=6, enc_depths=(1, 1), enc_channels=(32, 64), enc_num_head=(2, 4),
                              enc_patch_size=(16, 16), dec_depths=(1,), dec_channels=(32,), dec_num_head=(2,),
                              dec_patch_size=(16,), stride=(2,))


def test_failing_forward_raises_once_and_model_recovers():
    m = small_model()
    good = FakeRead([5, 10, 15, 20])          # 4 order rows of 5 runs each: m = 5
    bad = FakeRead([5, 11, 16, 21])           # row 1 counts 6 runs
    m._deferred = [(good, 5, 3, 1), (bad, 5, 3, 2)]
    with pytest.raises(RuntimeError, match=r"forward 3, pooling 2"):
        m.check_deferred(wait=True)
    assert m._deferred == []                  # taken off before validation
    m.check_deferred(wait=True)               # no stale error on the next check
    m._deferred = [(FakeRead([7, 14, 21, 28]), 7, 4, 1)]
    m.check_deferred(wait=True)               # a later good forward passes


def test_pending_reads_stay_until_ready_or_waited():
    m = small_model()
    late = FakeRead([5, 10, 15, 20], ready=False)
    bad_late = FakeRead([4, 10, 15, 20], ready=False)
    m._deferred = [(late, 5, 1, 1), (bad_late, 5, 2, 1)]
    m.check_deferred(wait=False)              # nothing landed: nothing checked, nothing raised
    assert len(m._deferred) == 2 and late.gets == 0
    with pytest.raises(RuntimeError, match=r"forward 2, pooling 1"):
        m.check_deferred(wait=True)
    assert m._deferred == [] and late.gets == 1
