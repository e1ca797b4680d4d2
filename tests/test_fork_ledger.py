"""The host-side fork/join check run at the end of every graph capture (ops.ForkLedger):
every stream forked during the capture must be joined directly into the capture's origin
stream (constraint (1)).  Pure host logic on stand-in stream ids."""
import pytest

from scattennet_amd import ops


class _S:
    def __init__(self, i):
        self.cuda_stream = i


def test_joined_into_origin_passes():
    o, side, br = _S(1), _S(2), _S(3)
    led = ops.ForkLedger(o)
    led.fork(br, o, "branch")
    led.fork(side, br, "side")  # forked from the branch ...
    led.join(o, br)
    led.join(o, side)           # ... joined into the origin
    assert led.problems() == []
    led.check()


def test_unjoined_fork_is_reported():
    o, side = _S(1), _S(2)
    led = ops.ForkLedger(o)
    led.fork(side, o, "side")
    assert led.problems() == ["stream side forked but not joined back"]
    with pytest.raises(RuntimeError, match="not joined back"):
        led.check()


def test_join_into_a_forked_stream_is_reported():
    o, br, side = _S(1), _S(2), _S(3)
    led = ops.ForkLedger(o)
    led.fork(br, o, "branch")
    led.fork(side, br, "side")
    led.join(br, side)  # side -> branch -> origin: the pattern that crashed instantiation
    led.join(o, br)
    assert led.problems() == ["stream side joined into 0x2, not into the capture origin"]


def test_fork_after_its_join_needs_another_join():
    o, side = _S(1), _S(2)
    led = ops.ForkLedger(o)
    led.fork(side, o, "side")
    led.join(o, side)
    led.fork(side, o, "side")  # re-forked later in the step
    assert led.problems() == ["stream side forked but not joined back"]
    led.join(o, side)
    assert led.problems() == []


def test_module_level_recording_is_off_outside_a_capture():
    assert ops._LEDGER is None
    ops.note_fork(_S(2), _S(1))  # no ledger: a no-op
    led = ops.fork_ledger_begin(_S(1))
    ops.note_fork(_S(2), _S(1), "side")
    ops.note_join(_S(1), _S(2))
    assert ops.fork_ledger_end() is led and ops._LEDGER is None
