"""Host logic of the drivers' packet-interval grouping (qg._IntervalGroup):
which slot each PDE step's snapshot goes to, when the intervals are handed
to swrt_advance_intervals, and the slot swap that starts the next group —
on a recording stand-in for the context (no GPU)."""
from swraytracing_amd.qg import _IntervalGroup


class _Rec:
    def __init__(self):
        self.calls = []

    def advance_intervals(self, dts, nsub, save_every=0):
        self.calls.append(("advance", list(dts), nsub))

    def swap_slots(self, a, b):
        self.calls.append(("swap", a, b))


def test_groups_of_k_then_swap_last_to_slot0():
    rec = _Rec()
    g = _IntervalGroup(rec, rec, 4, 5)
    slots = []
    for i in range(10):
        slots.append(g.next_slot())
        g.add(0.1 * (i + 1))
    g.flush()
    assert slots == [1, 2, 3, 4, 1, 2, 3, 4, 1, 2]
    assert rec.calls == [("advance", [0.1, 0.2, 0.30000000000000004, 0.4], 5), ("swap", 0, 4),
                         ("advance", [0.5, 0.6000000000000001, 0.7000000000000001, 0.8], 5), ("swap", 0, 4),
                         ("advance", [0.9, 1.0], 5), ("swap", 0, 2)]


def test_flush_on_frame_and_k1_is_one_call_per_step():
    rec = _Rec()
    g = _IntervalGroup(rec, rec, 4, 2)
    for i in range(3):
        g.add(1.0)
    g.flush()  # a frame is due: the partial group goes now
    g.flush()  # nothing pending: no call
    assert rec.calls == [("advance", [1.0, 1.0, 1.0], 2), ("swap", 0, 3)]
    rec1 = _Rec()
    g1 = _IntervalGroup(rec1, rec1, 1, 2)
    for _ in range(2):
        assert g1.next_slot() == 1
        g1.add(0.5)
    assert rec1.calls == [("advance", [0.5], 2), ("swap", 0, 1)] * 2


def test_group_size_is_clamped_to_the_slots():
    assert _IntervalGroup(None, None, 9, 1).k == 4
    assert _IntervalGroup(None, None, 0, 1).k == 1
