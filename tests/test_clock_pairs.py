"""The observed-shader-clock arithmetic (swrt_clock_ghz's pairing, host code in
swraytracing_amd/csrc/swrt_clock.cpp) on synthetic probe stamps, and bench.py's
handling of a clock that could not be observed — CPU only.

Round 5's two-rank bench test lost rank 1 in the fma_gather phase once, with
rank 0 then dying on the gloo all_reduce.  The only error path a phase's
timing had that the metric phase had survived is swrt_clock_ghz: two ranks
share GPU 0 there, the other rank's kernels hold the CUs while the probe
waves run, and when the start and end probes of one rank land on disjoint CUs
no CU holds both stamps — swrt_clock_ghz returns SWRT_ERR_STATE.  These tests
pin both halves: the pairing returns that error for disjoint CU sets (and only
then), and bench.timed turns it into an unobserved clock (None, None) instead
of a failed rank."""
import types

import numpy as np
import pytest

from swraytracing_amd._lib import SwrtError, clock_ghz_stamps


def _stamps(start_cus, end_cus, ghz, t0=1_000_000, dt_ticks=50_000, rt_hz=100e6, jitter=None):
    """Waves on the given CU ids: start stamps at realtime t0 (+ a wave index
    offset), end stamps dt_ticks later; each CU's cycle counter runs at
    ghz[cu] from its own arbitrary origin."""
    rng = np.random.default_rng(0)
    origin = {cu: int(rng.integers(0, 1 << 40)) for cu in set(start_cus) | set(end_cus)}
    w = max(len(start_cus), len(end_cus))
    a = np.zeros((2, w, 3), dtype=np.uint64)
    for side, cus, base in ((0, start_cus, t0), (1, end_cus, t0 + dt_ticks)):
        for i in range(w):
            cu = cus[i % len(cus)]
            rt = base + (i if side == 0 else -i)  # later start waves / earlier end waves on repeats
            cyc = origin[cu] + int(round(rt / rt_hz * ghz[cu] * 1e9))
            a[side, i] = (cyc, rt, cu)
    return a


def test_same_cu_pairs_give_the_median_clock():
    ghz = {c: 2.0 + 0.01 * c for c in range(8)}
    g, spread = clock_ghz_stamps(_stamps(list(range(8)), list(range(8)), ghz))
    assert abs(g - 2.04) < 1e-3  # the upper median of the 8 CU clocks (sorted[4])
    assert 0.0 <= spread < 0.05


def test_first_start_and_last_end_of_a_cu_are_paired():
    """Several waves per CU: the clock spans the CU's earliest start and latest
    end stamp (the widest interval), whatever the wave order."""
    ghz = {0: 1.7, 1: 1.7}
    a = _stamps([0, 1, 0, 1, 0, 1], [1, 0, 1, 0, 1, 0], ghz)
    g, _ = clock_ghz_stamps(a)
    assert abs(g - 1.7) < 1e-3


def test_disjoint_start_and_end_cus_have_no_clock():
    """The rank-abort case: start probes and end probes on disjoint CUs."""
    ghz = {c: 2.0 for c in range(8)}
    with pytest.raises(SwrtError, match="no CU with both"):
        clock_ghz_stamps(_stamps([0, 1, 2, 3], [4, 5, 6, 7], ghz))
    # one shared CU is enough
    g, _ = clock_ghz_stamps(_stamps([0, 1, 2, 3], [3, 5, 6, 7], ghz))
    assert abs(g - 2.0) < 1e-3


def test_bench_timed_reports_an_unobserved_clock(monkeypatch):
    """bench.timed with a context whose clock_ghz raises SwrtError (no CU ran
    both probe waves) returns clk = (None, None) and completes."""
    import bench
    bench._imports()
    monkeypatch.setattr(bench.torch.cuda, "synchronize", lambda *a, **k: None)
    calls = []

    class StubCtx:
        def synchronize(self):
            calls.append("sync")

        def set_timing(self, every):
            calls.append(("timing", every))

        def kernel_time(self, reset=True):
            return 1.5, 3

        def clock_stamp(self, which):
            calls.append(("stamp", which))

        def clock_ghz(self):
            raise bench.sw.SwrtError("swrt_clock_ghz: SWRT_ERR_STATE: no CU with both a start and an end stamp")

        def advance(self, *a, **k):
            calls.append("advance")

    w = {"dt": 0.01, "f": 3.0, "gH": 1.0, "nslots": 2, "intervals": 1}
    args = types.SimpleNamespace(substeps=5, timing_every=5)
    el, kms, launches, clk = bench.timed(StubCtx(), w, args, None, steps=3, warmup=1)
    assert clk == (None, None)
    assert (kms, launches) == (1.5, 3) and el >= 0
    assert calls.count("advance") == 4 and ("stamp", 0) in calls and ("stamp", 1) in calls
