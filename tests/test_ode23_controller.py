"""The library's ode23 controller (swrt_ode23_ctl.cpp, the code swrt_ode23_run
runs) against swraytracing_amd/integrate.py's controller, on the CPU.

MATLAB's ode23 step-size logic (qgsw_raytrace.m:149, qg2layersw_raytrace.m:195)
exists twice in this repo: in C++ inside libswrt, where it drives the device
stages with speculative next attempts, gated guesses and the device's own
first step, and in Python, where it drives the sharded ensemble through the
error norm's allreduce.  Both are fed the same scripted raw-error sequences
here (no GPU: swrt_ode23_replay runs the C++ controller over a script instead
of the device), covering rejected attempts, hmin, the clamp to tfinal and all
three guess gates; the consumed attempts (t, h, tnew), the accepted times and
the counts must agree bit for bit.  MATLAB's own ode23 is not available:
parity with it is unpinned, the restatement is what is pinned."""
import math

import numpy as np
import pytest

from swraytracing_amd._lib import ode23_replay
from swraytracing_amd.integrate import ode23_packets


class _Script:
    """A stand-in for the device stages: raw maxima from an error model of
    the attempt (t, h, tnew), recorded in the order the controller asks."""

    def __init__(self, model):
        self.model = model
        self.raws = []
        self.attempts = []
        self.accepts = 0

    def ode23_f1(self, t, tmax, f, Cg, nslots, thr, bump):
        r = float(self.model("f1", t, 0.0, 0.0, len(self.attempts)))
        self.raws.append(r)
        return r

    def ode23_attempt(self, t, h, tnew, tmax, f, Cg, nslots, thr, bump):
        r = float(self.model("attempt", t, h, tnew, len(self.attempts)))
        self.raws.append(r)
        self.attempts.append((t, h, tnew, r))
        return r

    def ode23_accept(self):
        self.accepts += 1


def _third_order(C, rh=50.0):
    """err = C*|h|^3 (a smooth 3rd-order local error): raw = err/absh."""
    return lambda kind, t, h, tnew, i: rh if kind == "f1" else C * abs(h) ** 2


def _random(seed, lo=-7.0, hi=1.5):
    """err spread log-uniformly over [10^lo, 10^hi]*rtol: accepts, rejections
    and every ramp-up rule in one run."""
    rng = np.random.default_rng(seed)
    return lambda kind, t, h, tnew, i: (10.0 ** rng.uniform(0, 3) if kind == "f1"
                                        else 1e-3 * 10.0 ** rng.uniform(lo, hi) / abs(h))


def _reject_every(k, C):
    """A smooth model with every k-th attempt rejected outright."""
    def m(kind, t, h, tnew, i):
        if kind == "f1":
            return 20.0
        return 1e3 / abs(h) if i % k == k - 1 else C * abs(h) ** 2
    return m


def _always_reject(kind, t, h, tnew, i):
    return 5.0 if kind == "f1" else 1e300  # never accepted: down to hmin


CASES = {
    "third_order_small": (_third_order(1e-2), 0.0, 0.0125),
    "third_order_mid": (_third_order(2e2), 0.0, 0.0125),
    "third_order_large": (_third_order(5e6), 0.0, 0.0125),
    "random_a": (_random(1), 0.0, 0.0125),
    "random_b": (_random(2, -5.0, 0.8), 1.0, 1.0125),
    "random_reverse": (_random(3), 0.5, 0.375),
    "reject_every_4": (_reject_every(4, 3e3), 0.0, 0.02),
    "reject_every_3": (_reject_every(3, 1e1), 0.0, 0.02),
}


def _run_python(model, t0, tfinal):
    ctx = _Script(model)
    st = {}
    try:
        ts = ode23_packets(ctx, (t0, tfinal), tfinal, 3.0, 1.0, controller="python", stats=st)
        status = 0
    except RuntimeError as e:
        assert "below hmin" in str(e)
        ts, status = None, "below hmin"
    return ctx, ts, st, status


@pytest.mark.parametrize("dev_first", [True, False])
@pytest.mark.parametrize("name", sorted(CASES))
def test_library_controller_takes_the_python_controllers_steps(name, dev_first):
    model, t0, tfinal = CASES[name]
    ctx, ts, st, status = _run_python(model, t0, tfinal)
    rc, log, ts_c, stc = ode23_replay(t0, tfinal, ctx.raws, dev_first=dev_first)
    assert rc == status == 0
    want = np.array(ctx.attempts, dtype=np.float64).reshape(-1, 4)
    assert log.shape == want.shape
    assert np.array_equal(log.view(np.uint64), want.view(np.uint64)), "consumed attempts differ"
    assert np.array_equal(ts_c.view(np.uint64), np.asarray(ts, dtype=np.float64).view(np.uint64))
    assert (stc["steps"], stc["failed"], stc["attempts"]) == (st["steps"], st["failed"], st["attempts"])
    assert ctx.accepts == stc["steps"]
    assert stc["gate_violations"] == 0  # no consumed guess the device gate would have skipped
    assert ts_c[-1] == tfinal  # the clamp to tfinal
    assert stc["first_taken"] == (1 if dev_first else 0)


def test_below_hmin_fails_at_the_same_attempt():
    for dev_first in (True, False):
        # (t0 = 1: hmin = 16*spacing(1) ~ 3.6e-15 is reached after ~40 halvings)
        ctx, ts, st, status = _run_python(_always_reject, 1.0, 1.01)
        rc, log, ts_c, stc = ode23_replay(1.0, 1.01, ctx.raws, dev_first=dev_first)
        assert status == rc == "below hmin"
        want = np.array(ctx.attempts, dtype=np.float64).reshape(-1, 4)
        assert np.array_equal(log.view(np.uint64), want.view(np.uint64))
        assert stc["attempts"] == len(ctx.attempts) and stc["failed"] == len(ctx.attempts)
        assert list(ts_c) == [1.0]  # nothing accepted
        assert stc["gate_violations"] == 0


def test_every_guess_gate_is_taken_across_the_cases():
    """The three guess rules (MaxStep at MaxStep, MaxStep from 5*absh, 5*absh)
    each save a host round trip somewhere in the scripted cases, and every
    rejection path (first failure's pow rule, then halving) is exercised."""
    taken = {"taken_maxstep": 0, "taken_ramp_maxstep": 0, "taken_ramp_5x": 0}
    failed = 0
    multi_fail = False
    for name, (model, t0, tfinal) in CASES.items():
        ctx, _, st, _ = _run_python(model, t0, tfinal)
        _, log, _, stc = ode23_replay(t0, tfinal, ctx.raws)
        for k in taken:
            taken[k] += stc[k]
        failed += stc["failed"]
        # two rejections in a row at one t: the halving branch
        t = log[:, 0]
        multi_fail |= bool(np.any((t[1:] == t[:-1]) & (np.r_[t[2:], np.nan] == t[1:])))
    assert all(v > 0 for v in taken.values()), taken
    assert failed > 0 and multi_fail


def test_script_exhausted_is_reported():
    ctx, _, _, _ = _run_python(_third_order(1e-2), 0.0, 0.0125)
    rc, _, _, _ = ode23_replay(0.0, 0.0125, ctx.raws[:-1])
    assert rc == "script exhausted"


def test_driver_like_interval_steps():
    """The drivers' interval [0, dt] with MaxStep 0.1*dt: a smooth error small
    enough that every step is MaxStep after the ramp-up, as in the bench's
    ode23 intervals (~13 attempts, none rejected)."""
    dt = 0.0123
    ctx, ts, st, _ = _run_python(_third_order(1e-4, rh=80.0), 0.0, dt)
    rc, log, ts_c, stc = ode23_replay(0.0, dt, ctx.raws)
    assert rc == 0 and stc["failed"] == 0
    assert np.array_equal(ts_c, ts)
    hs = np.diff(ts_c)
    assert math.isclose(hs[-2], 0.1 * dt, rel_tol=1e-12)
    assert stc["taken_maxstep"] > 0
