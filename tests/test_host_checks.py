"""Host-side guards of the product path (no GPU needed).

* `_lib.check_lookback`: a decoupled look-back wait that reached its spin cap (csrc/common.h lb_lookback_wave)
  makes the scan's prefix wrong; the consumers (FeaturePredictor.check_refine, evaluate_scenes, Trainer.micro_step,
  bench.py after the timed steps) call the check, which raises once per new timeout and names the caller.
* `ptv3_train.DropMasks`: the DropPath hash seeds differ per rank and per mask source, advance per draw, and
  survive a state_dict round trip (a resumed Trainer does not replay step 0's masks).
"""
import pytest

from splatformer_amd import _lib
from splatformer_amd import ptv3_train as pt


def test_lookback_timeout_raises_once(monkeypatch):
    counts = iter([0, -1, 0, 2, 2, 2, 3])

    def fake(_stream):
        return next(counts)

    monkeypatch.setattr(_lib, "fn", lambda name: fake if name == "sfx_lookback_timeouts" else None)
    monkeypatch.setattr(_lib, "_LB_SEEN", {})
    st = 12345
    _lib.check_lookback("a", st)            # 0: exact
    _lib.check_lookback("b", st)            # -1: nothing scanned yet
    _lib.check_lookback("c", st)            # 0
    with pytest.raises(RuntimeError, match=r"^bench: 2 decoupled look-back"):
        _lib.check_lookback("bench", st)    # 2 new timeouts: raised once
    _lib.check_lookback("d", st)            # still 2: already reported
    _lib.check_lookback("e", st)
    with pytest.raises(RuntimeError, match=r"^Trainer\.micro_step: 1 decoupled"):
        _lib.check_lookback("Trainer.micro_step", st)  # one more


def test_drop_masks_seed_streams():
    a0 = pt.DropMasks(None, rank=0)
    a1 = pt.DropMasks(None, rank=1)
    b0 = pt.DropMasks(None, rank=0)       # a second source on the same rank (a re-created Trainer)
    assert a0.base == a1.base == b0.base
    assert len({a0.seed(), a1.seed(), b0.seed()}) == 3
    s0 = a0.seed()
    a0.k += 1
    assert a0.seed() != s0
    sd = a0.state_dict()
    c = pt.DropMasks(None, rank=5)
    c.load_state_dict(sd)
    assert c.seed() == a0.seed() and c.state_dict() == sd
    # p == 0 is Identity: no draw, no device work
    assert a0("x", 10, 0.0) is None and a0.k == sd["k"]
