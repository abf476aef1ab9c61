"""GPU ode23 (swrt_ode23_* stages + the controller, in the library (swrt_ode23_run)
or in Python (ode23_packets)) against
the oracle's restatement of MATLAB ode23 with the drivers' odefun
(qgsw_raytrace.m:143-150,259-265).  Every stage is the same IEEE-754 op
sequence as the oracle (same stencil code, correctly rounded sqrt/division,
-ffp-contract=off) and the error norm is a max, so the step sequence and the
final state are bit-identical.  (MATLAB's own ode23 is not pinned.)"""
import numpy as np
import pytest

import swraytracing_amd as sw
from oracle import swrt_oracle as orc
from tests.test_gpu_parity import _planes

pytestmark = pytest.mark.gpu


def _y0(x, k):
    return np.concatenate([x[:, 0], x[:, 1], k[:, 0], k[:, 1]])


@pytest.mark.parametrize("controller", ["library", "python"])
@pytest.mark.parametrize("rebin", [0, 4])
def test_ode23_packets_bitexact(ctx, qg_case, rebin, controller):
    c = qg_case
    nx, L, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    flow1 = c["flow"]
    flow2 = {n: np.asarray(v) * 1.3 for n, v in flow1.items()}
    ctx.set_field_grid(0, _planes(flow1), nx, L)
    ctx.set_field_grid(1, _planes(flow2), nx, L)
    x, k = c["x"][:200], c["k"][:200]
    tmax = 40 * c["dt"]  # long enough for several (and some rejected) steps
    ctx.set_locality(rebin, 0)
    try:
        ctx.packets_set(x, k)
        st = {}
        ts = sw.ode23_packets(ctx, (0.0, tmax), tmax, f, Cg, stats=st, controller=controller)
        xg, kg = ctx.packets_get()
    finally:
        ctx.set_locality(4, 0)
    rhs = orc.raytracing_rhs(flow1, flow2, f, Cg, tmax, L / nx)
    so = {}
    to, yo = orc.ode23(rhs, [0.0, tmax], _y0(x, k), stats=so)
    n = x.shape[0]
    np.testing.assert_array_equal(ts, to)
    assert so["failed"] > 0 and so["steps"] > 10
    assert st["steps"] == so["steps"] and st["failed"] == so["failed"]
    np.testing.assert_array_equal(xg[:, 0], yo[:n])
    np.testing.assert_array_equal(xg[:, 1], yo[n:2 * n])
    np.testing.assert_array_equal(kg[:, 0], yo[2 * n:3 * n])
    np.testing.assert_array_equal(kg[:, 1], yo[3 * n:])


@pytest.mark.parametrize("controller", ["library", "python"])
def test_ode23_rejections_happen_and_match(ctx, qg_case, controller):
    """A loose start (tiny rtol) forces rejected steps; still bit-identical
    (the controller in the library, swrt_ode23_run, or the Python loop)."""
    c = qg_case
    nx, L, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    flow1 = c["flow"]
    flow2 = {n: np.asarray(v) * -0.7 for n, v in flow1.items()}
    ctx.set_field_grid(0, _planes(flow1), nx, L)
    ctx.set_field_grid(1, _planes(flow2), nx, L)
    x, k = c["x"][:64], c["k"][:64] * 4
    tmax = 60 * c["dt"]
    ctx.packets_set(x, k)
    st = {}
    ts = sw.ode23_packets(ctx, (0.0, tmax), tmax, f, Cg, rtol=1e-6, atol=1e-9, stats=st, controller=controller)
    xg, kg = ctx.packets_get()
    so = {}
    to, yo = orc.ode23(orc.raytracing_rhs(flow1, flow2, f, Cg, tmax, L / nx), [0.0, tmax], _y0(x, k),
                       rtol=1e-6, atol=1e-9, stats=so)
    np.testing.assert_array_equal(ts, to)
    assert so["failed"] > 0
    assert st["failed"] == so["failed"]
    np.testing.assert_array_equal(np.concatenate([xg[:, 0], xg[:, 1], kg[:, 0], kg[:, 1]]), yo)


def test_ode23_run_ts_cap_bounds_times_only(ctx, qg_case):
    """A ts_cap smaller than the step count truncates the recorded times; the
    interval still completes with the full-cap state."""
    c = qg_case
    nx, L, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    ctx.set_field_grid(0, _planes(c["flow"]), nx, L)
    ctx.set_field_grid(1, _planes({n: np.asarray(v) * 1.3 for n, v in c["flow"].items()}), nx, L)
    x, k = c["x"][:128], c["k"][:128]
    tmax = 40 * c["dt"]
    out = []
    for cap in (100_000, 3):
        ctx.packets_set(x, k)
        if cap < 100:  # fewer slots than accepted times: the caller is told
            with pytest.warns(RuntimeWarning, match="accepted"):
                ts, st = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG, ts_cap=cap)
        else:
            ts, st = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG, ts_cap=cap)
        out.append((ts, st, *ctx.packets_get()))
    (ts_a, st_a, xa, ka), (ts_b, st_b, xb, kb) = out
    assert st_a == st_b and st_a["steps"] > 3 and st_a["accepted"] == len(ts_a) > 3
    np.testing.assert_array_equal(ts_b, ts_a[:3])
    np.testing.assert_array_equal(xb, xa)
    np.testing.assert_array_equal(kb, ka)


def test_packet_ensemble_ode23_interval(ctx, qg_case):
    """PacketEnsemble.advance_ode23 == ode23(ray_ode, [0, dt], y0) with the
    snapshots in slots 0/1 (the drivers' packet branch)."""
    c = qg_case
    nx, L, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    ens = sw.PacketEnsemble(c["x"], c["k"], L, f, Cg, nx, c["K_d2"], ctx=ctx)
    q2 = c["qk"] * np.exp(0.1j)
    ens.set_snapshots(c["qk"], q2)
    dt = 25 * c["dt"]
    ens.advance_ode23(dt)
    xg, kg = ens.state()
    p0 = ctx.get_field_grid(0, nx)
    p1 = ctx.get_field_grid(1, nx)
    fl = lambda p: {n: p[i].reshape((nx, nx), order="F") for i, n in enumerate(orc.FIELD_ORDER)}
    to, yo = orc.ode23(orc.raytracing_rhs(fl(p0), fl(p1), f, Cg, dt, L / nx), [0.0, dt], _y0(c["x"], c["k"]))
    n = c["x"].shape[0]
    np.testing.assert_array_equal(np.concatenate([xg[:, 0], xg[:, 1], kg[:, 0], kg[:, 1]]), yo)


def test_golden_ode23_fixture(ctx):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_ode23.npz"))
    nx, L = int(g["nx"]), float(g["L"])
    ctx.set_field_grid(0, g["planes0"], nx, L, int(g["ny_period"]))
    ctx.set_field_grid(1, g["planes1"], nx, L, int(g["ny_period"]))
    ctx.packets_set(g["x0"], g["k0"])
    ts = sw.ode23_packets(ctx, (0.0, float(g["tmax"])), float(g["tmax"]), float(g["f"]), float(g["Cg"]))
    xg, kg = ctx.packets_get()
    np.testing.assert_array_equal(ts, g["ts"])
    np.testing.assert_array_equal(np.concatenate([xg[:, 0], xg[:, 1], kg[:, 0], kg[:, 1]]), g["y"])


@pytest.mark.parametrize("hz", [0, 1])
def test_ode23_run_split_attempts_match_python_controller(ctx, qg_case, hz):
    """70,000 packets on 16 tiles: swrt_ode23_run splits every attempt into
    two part launches on the two packet streams, reads the error max from the
    workgroups' host-mapped maxima (no copy between attempts) and queues a
    gated guess of the next attempt through the ramp-up (5*absh) as well as at
    MaxStep — the same steps and bits as the Python controller's one launch
    and copied max per attempt.  With the hazard checker on (hz) the mapped
    maxima are also checked against the device's atomicMax slots."""
    from swraytracing_amd import _lib as L
    c = qg_case
    nx, Lx, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    flow1 = c["flow"]
    flow2 = {n: np.asarray(v) * 1.3 for n, v in flow1.items()}
    ctx.set_field_grid(0, _planes(flow1), nx, Lx)
    ctx.set_field_grid(1, _planes(flow2), nx, Lx)
    rng = np.random.default_rng(23)
    n = 70_000
    x = rng.uniform(-Lx / 2, Lx / 2, (n, 2))
    k = c["k"][rng.integers(0, c["k"].shape[0], n)]
    tmax = 40 * c["dt"]
    ctx.set_locality(4, 0)
    outs = []
    try:
        for controller in ("python", "library"):
            ctx.debug_set(L.DEBUG_HAZARD_CHECK, hz if controller == "library" else 0)
            ctx.packets_set(x, k)
            st = {}
            ts = sw.ode23_packets(ctx, (0.0, tmax), tmax, f, Cg, stats=st, controller=controller)
            outs.append((ts, st, *ctx.packets_get()))
    finally:
        ctx.debug_set(L.DEBUG_HAZARD_CHECK, 0)
    (ts_p, st_p, xp, kp), (ts_l, st_l, xl, kl) = outs
    assert st_l["steps"] > 5
    np.testing.assert_array_equal(ts_l, ts_p)
    assert (st_l["steps"], st_l["failed"], st_l["attempts"]) == (st_p["steps"], st_p["failed"], st_p["attempts"])
    np.testing.assert_array_equal(xl, xp)
    np.testing.assert_array_equal(kl, kp)


def test_ode23_run_hook_runs_once_and_its_exception_surfaces(ctx, qg_case):
    """swrt_ode23_run_hooked calls the hook once, after the interval's first
    launches are queued; an exception the hook raises reaches the caller after
    the interval completes, with the packets advanced exactly as without a
    hook (the hook may only queue other work)."""
    c = qg_case
    nx, L, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    ctx.set_field_grid(0, _planes(c["flow"]), nx, L)
    ctx.set_field_grid(1, _planes({n: np.asarray(v) * 1.3 for n, v in c["flow"].items()}), nx, L)
    x, k = c["x"][:128], c["k"][:128]
    tmax = 20 * c["dt"]
    ctx.packets_set(x, k)
    ts0 = sw.ode23_packets(ctx, (0.0, tmax), tmax, f, Cg)
    x0, k0 = ctx.packets_get()
    calls = []
    ctx.packets_set(x, k)
    ts1 = sw.ode23_packets(ctx, (0.0, tmax), tmax, f, Cg, hook=lambda: calls.append(1))
    assert calls == [1]
    np.testing.assert_array_equal(ts1, ts0)

    def bad():
        raise ValueError("hook failed")
    ctx.packets_set(x, k)
    with pytest.raises(ValueError, match="hook failed"):
        sw.ode23_packets(ctx, (0.0, tmax), tmax, f, Cg, hook=bad)
    x2, k2 = ctx.packets_get()
    np.testing.assert_array_equal(x2, x0)
    np.testing.assert_array_equal(k2, k0)


def test_ode23_chain_taken_only_when_exact(ctx, qg_case):
    """swrt_ode23_chain_next: an ode23 call queues the next call's stage 1
    (f at t = 0 on its accepted packets, the armed slots as slots 0 / 1) as
    it ends; the next call takes it only when it computes exactly that.  Two
    chained intervals (the drivers' slot rotation between them) against the
    same two unchained: the same times and packet bits whether the chain is
    taken (plain, with the hazard checker modelling its launches, and for an
    interval of another length: alpha(0) = 0 all the same) or dropped — by a
    rewrite of a slot it read (even with the same data), by a call that may
    touch the packets, or by another RelTol.  Behind its stage 1 the chain
    also queues the next call's first step size and first (split) attempt;
    that call takes them only for the t0, tfinal and RelTol they assumed
    (DEBUG_ODE23_FIRST_CHAINED), else joins and discards them."""
    from swraytracing_amd import _lib as L
    c = qg_case
    nx, Lx, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    flows = [c["flow"]] + [{n: np.asarray(v) * s for n, v in c["flow"].items()} for s in (1.3, -0.7)]
    rng = np.random.default_rng(29)
    n = 70_000  # two part launches per attempt (the split) on 16 tiles
    x = rng.uniform(-Lx / 2, Lx / 2, (n, 2))
    k = c["k"][rng.integers(0, c["k"].shape[0], n)]
    tmax = 30 * c["dt"]
    bump = orc.BUMP_QG

    def run(arm, between=None, rtol2=1e-3, tfinal2=tmax, hz=0, rtol1=1e-3, tmax2=tmax):
        for s in range(3):
            ctx.set_field_grid(s, _planes(flows[s]), nx, Lx)
        ctx.debug_set(L.DEBUG_HAZARD_CHECK, hz)
        try:
            ctx.packets_set(x, k)
            n0 = ctx.debug_get(L.DEBUG_ODE23_CHAINED)
            f0 = ctx.debug_get(L.DEBUG_ODE23_FIRST_CHAINED)
            hook = (lambda: ctx.ode23_chain_next(1, 2)) if arm else None
            ts1, _ = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, rtol1, 1e-6, bump, hook=hook)
            ctx.swap_slots(0, 1)
            ctx.swap_slots(1, 2)  # the armed slots 1 / 2 are now slots 0 / 1
            if between is not None:
                between()
            ts2, st2 = ctx.ode23_run(0.0, tfinal2, tmax2, f, Cg, 2, rtol2, 1e-6, bump)
            taken = ctx.debug_get(L.DEBUG_ODE23_CHAINED) - n0
            first = ctx.debug_get(L.DEBUG_ODE23_FIRST_CHAINED) - f0
            return ts1, ts2, *ctx.packets_get(), taken, st2, first
        finally:
            ctx.debug_set(L.DEBUG_HAZARD_CHECK, 0)

    ctx.set_locality(4, 0)

    def same(a, b):
        for u, v in zip(a[:4], b[:4]):
            np.testing.assert_array_equal(u, v)
        assert a[5] == b[5]  # steps, failed, attempts of the second interval

    ref = run(False)
    assert ref[4] == 0 and ref[6] == 0 and len(ref[0]) > 5 and len(ref[1]) > 5
    for hz in (0, 1):
        chained = run(True, hz=hz)
        assert chained[4] == 1 and chained[6] == 1
        same(chained, ref)
    # a host synchronisation between the calls keeps the chain (and ends part 1)
    synced = run(True, between=ctx.synchronize)
    assert synced[4] == 1 and synced[6] == 1
    same(synced, ref)
    rewrite = run(True, between=lambda: ctx.set_field_grid(1, _planes(flows[2]), nx, Lx))
    assert rewrite[4] == 0 and rewrite[6] == 0
    same(rewrite, ref)
    touched = run(True, between=lambda: ctx.packets_get())
    assert touched[4] == 0 and touched[6] == 0
    same(touched, ref)
    # another RelTol: another stage-1 input (AbsTol/RelTol), dropped
    other = run(True, rtol2=1e-4)
    assert other[4] == 0 and other[6] == 0
    same(other, run(False, rtol2=1e-4))
    # tight tolerances: rejected attempts in both intervals, chain taken
    tight = run(True, rtol1=1e-7, rtol2=1e-7)
    assert tight[4] == 1 and tight[6] == 1 and tight[5]["failed"] > 0
    same(tight, run(False, rtol1=1e-7, rtol2=1e-7))
    # another interval length (same tmax, t0 = 0): the same stage 1, taken;
    # the first attempt assumed tfinal = tmax: joined and discarded
    half = run(True, tfinal2=0.5 * tmax)
    assert half[4] == 1 and half[6] == 0
    same(half, run(False, tfinal2=0.5 * tmax))
    # the same tfinal over another tmax (the attempt's alpha = t / tmax): stage
    # 1 taken (alpha(0) = 0), the first attempt discarded
    longer = run(True, tmax2=2 * tmax)
    assert longer[4] == 1 and longer[6] == 0
    same(longer, run(False, tmax2=2 * tmax))


def test_ode23_driver_path_at_scale_matches_oracle(fresh_ctx, qg_case, oracle_lib):
    """The library ode23 path exactly as the drivers run it (qgsw_raytrace.m:
    143-150, qg2layersw_raytrace.m:195-196), against the oracle's ode23 rather
    than against the Python controller: 70,000 packets on 16 tiles so every
    attempt is split into two part launches (ode23_split_ok), maxima read from
    host-mapped memory, the first attempt queued from the device's own step
    size, gated guesses, and two intervals chained (the second one's stage 1
    queued by the first as it ends, the drivers' slot rotation between them).
    The events are asserted to have happened; times, step counts and the
    final packet bits equal orc.ode23 over the same two intervals (its odefun
    through the C oracle's interpolation, checked bit-identical to the numpy
    restatement first)."""
    from oracle import cbind
    from swraytracing_amd import _lib as L
    ctx = fresh_ctx
    c = qg_case
    nx, Lx, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    flows = [c["flow"]] + [{n: np.asarray(v) * s for n, v in c["flow"].items()} for s in (1.3, -0.7)]
    planes = [_planes(fl) for fl in flows]
    rng = np.random.default_rng(31)
    n = 70_000
    x = rng.uniform(-Lx / 2, Lx / 2, (n, 2))
    k = c["k"][rng.integers(0, c["k"].shape[0], n)]
    tmax = 40 * c["dt"]  # MaxStep 4 dt: the controller rejects some steps at the default tolerances
    bump = orc.BUMP_QG
    keys = (L.DEBUG_ODE23_CHAINED, L.DEBUG_ODE23_FIRST_TAKEN, L.DEBUG_ODE23_GUESSES_TAKEN, L.DEBUG_ODE23_SPLIT_RUNS,
            L.DEBUG_ODE23_FIRST_CHAINED)
    ctx.set_locality(4, 0)
    for s in range(3):
        ctx.set_field_grid(s, planes[s], nx, Lx)
    ctx.packets_set(x, k)
    before = [ctx.debug_get(key) for key in keys]
    ts1, st1 = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, bump, hook=lambda: ctx.ode23_chain_next(1, 2))
    ctx.swap_slots(0, 1)
    ctx.swap_slots(1, 2)  # the armed slots 1 / 2 are now slots 0 / 1
    ts2, st2 = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, bump)
    xg, kg = ctx.packets_get()
    chained, first, guesses, split, first_chained = [ctx.debug_get(key) - b for key, b in zip(keys, before)]
    assert split == 2 and first == 2 and chained == 1 and first_chained == 1, (split, first, chained, first_chained)
    assert guesses >= 1 and st1["failed"] + st2["failed"] >= 1, (guesses, st1, st2)
    dx = Lx / nx
    rhs = [cbind.raytracing_rhs(planes[i], planes[i + 1], f, Cg, tmax, nx, nx, dx, bump) for i in (0, 1)]
    sub = _y0(x[:3000], k[:3000])
    for i, t in ((0, 0.0), (1, 0.37 * tmax)):
        np.testing.assert_array_equal(rhs[i](t, sub), orc.raytracing_rhs(flows[i], flows[i + 1], f, Cg, tmax, dx)(t, sub))
    so1, so2 = {}, {}
    to1, y1 = orc.ode23(rhs[0], [0.0, tmax], _y0(x, k), stats=so1)
    to2, y2 = orc.ode23(rhs[1], [0.0, tmax], y1, stats=so2)
    np.testing.assert_array_equal(ts1, to1)
    np.testing.assert_array_equal(ts2, to2)
    assert (st1["steps"], st1["failed"]) == (so1["steps"], so1["failed"])
    assert (st2["steps"], st2["failed"]) == (so2["steps"], so2["failed"])
    np.testing.assert_array_equal(np.concatenate([xg[:, 0], xg[:, 1], kg[:, 0], kg[:, 1]]), y2)


def test_ode23_hook_may_not_touch_the_packets(fresh_ctx, qg_case):
    """A hook that calls an entry point that may touch the packets (packets_set,
    advance, packets_get, another ode23 call) is refused with SWRT_ERR_STATE
    (it would race the interval's attempts in flight); the interval itself
    completes with the bits of a hook-free run.  QG-stream calls and
    swrt_ode23_chain_next stay allowed (the drivers' hook)."""
    ctx = fresh_ctx
    c = qg_case
    nx, L, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    ctx.set_field_grid(0, _planes(c["flow"]), nx, L)
    ctx.set_field_grid(1, _planes({n: np.asarray(v) * 1.3 for n, v in c["flow"].items()}), nx, L)
    rng = np.random.default_rng(5)
    n = 70_000
    x = rng.uniform(-L / 2, L / 2, (n, 2))
    k = c["k"][rng.integers(0, c["k"].shape[0], n)]
    tmax = 20 * c["dt"]
    ctx.set_locality(4, 0)
    ctx.packets_set(x, k)
    ts0, _ = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG)
    x0, k0 = ctx.packets_get()
    bad = {
        "packets_set": lambda: ctx.packets_set(x, k),
        "advance": lambda: ctx.advance(1e-3, 1, f, 1.0, nslots=2, bump=orc.BUMP_QG),
        "packets_get": ctx.packets_get,
        "ode23_run": lambda: ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG),
    }
    for name, call in bad.items():
        ctx.packets_set(x, k)
        with pytest.raises(sw.SwrtError, match="SWRT_ERR_STATE"):
            ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG, hook=call)
        x1, k1 = ctx.packets_get()
        np.testing.assert_array_equal(x1, x0, err_msg=name)
        np.testing.assert_array_equal(k1, k0, err_msg=name)
    ctx.packets_set(x, k)
    ts2, _ = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG, hook=lambda: ctx.ode23_chain_next(0, 1))
    np.testing.assert_array_equal(ts2, ts0)


def test_ode23_chain_dropped_by_a_qg_snapshot_rewrite(fresh_ctx, qg_case):
    """swrt_qg_snapshot keeps a queued chain (it never touches the packets), so
    the chain's own check — the slots hold the same nodes, not rewritten
    since (write generation) — is what drops it when a snapshot rewrites a
    slot it read, even with identical data (the drivers' CFL-rejection path).
    The bits then equal the unchained run's."""
    from swraytracing_amd import _lib as L
    ctx = fresh_ctx
    c = qg_case
    nx, Lx, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    model = sw.QGModel.one_layer(c["qk"], nx, f, Cg, ctx=ctx)
    model.step(c["dt"])
    model.snapshot(2)  # slot 2 = grid_U of the QG state's qk
    snap = ctx.get_field_grid(2, nx)
    flows = [_planes(c["flow"]), _planes({n: np.asarray(v) * 1.3 for n, v in c["flow"].items()}), snap]
    rng = np.random.default_rng(37)
    n = 70_000
    x = rng.uniform(-Lx / 2, Lx / 2, (n, 2))
    k = c["k"][rng.integers(0, c["k"].shape[0], n)]
    tmax = 30 * c["dt"]
    ctx.set_locality(4, 0)

    def run(arm, rewrite):
        for s in range(3):
            if s == 2:
                model.snapshot(2)
            else:
                ctx.set_field_grid(s, flows[s], nx, Lx)
        ctx.packets_set(x, k)
        n0 = ctx.debug_get(L.DEBUG_ODE23_CHAINED)
        hook = (lambda: ctx.ode23_chain_next(1, 2)) if arm else None
        ts1, _ = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG, hook=hook)
        ctx.swap_slots(0, 1)
        ctx.swap_slots(1, 2)
        if rewrite:
            model.snapshot(1)  # the same grid_U into the slot the chain read as its slot 1
        ts2, st2 = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, orc.BUMP_QG)
        return ts1, ts2, *ctx.packets_get(), ctx.debug_get(L.DEBUG_ODE23_CHAINED) - n0, st2

    ref = run(False, False)
    np.testing.assert_array_equal(ctx.get_field_grid(1, nx), snap)
    kept = run(True, False)
    assert kept[4] == 1
    dropped = run(True, True)
    assert dropped[4] == 0
    for a in (kept, dropped):
        for u, v in zip(a[:4], ref[:4]):
            np.testing.assert_array_equal(u, v)
        assert a[5] == ref[5]


def test_ode23_run_sharded_reduce_steps_and_bits(fresh_ctx, qg_case):
    """swrt_ode23_run_sharded (the library controller of a sharded run): with
    an identity reduce — one rank — the same times, counts and packet bits as
    swrt_ode23_run, though its first step size is not guessed on the device.
    The reduce is called once for stage 1 and once per attempt; a reduce that
    raises surfaces its exception."""
    ctx = fresh_ctx
    c = qg_case
    nx, Lx, f, Cg = c["nx"], c["L"], c["f"], c["Cg"]
    flows = [c["flow"], {n: np.asarray(v) * 1.3 for n, v in c["flow"].items()}]
    rng = np.random.default_rng(37)
    n = 70_000
    x = rng.uniform(-Lx / 2, Lx / 2, (n, 2))
    k = c["k"][rng.integers(0, c["k"].shape[0], n)]
    tmax = 30 * c["dt"]
    bump = orc.BUMP_QG
    ctx.set_locality(4, 0)
    for s in range(2):
        ctx.set_field_grid(s, _planes(flows[s]), nx, Lx)

    def run(reduce):
        ctx.packets_set(x, k)
        ts, st = ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, bump, reduce=reduce)
        return ts, st, *ctx.packets_get()

    calls = []

    def ident(v):
        calls.append(v)
        return v

    a = run(None)
    b = run(ident)
    np.testing.assert_array_equal(a[0], b[0])
    assert (a[1]["steps"], a[1]["failed"], a[1]["attempts"]) == (b[1]["steps"], b[1]["failed"], b[1]["attempts"])
    np.testing.assert_array_equal(a[2], b[2])
    np.testing.assert_array_equal(a[3], b[3])
    assert len(calls) == 1 + b[1]["attempts"] and all(v >= 0 for v in calls)

    def boom(v):
        raise KeyError("reduce failed on purpose")

    ctx.packets_set(x, k)
    with pytest.raises(KeyError, match="on purpose"):
        ctx.ode23_run(0.0, tmax, tmax, f, Cg, 2, 1e-3, 1e-6, bump, reduce=boom)


def test_ode23_driver_longer_run_same_files_with_and_without_chaining(tmp_path, monkeypatch):
    """The 2-layer driver with the reference's ode23 over 48 PDE steps (its
    CFL rule, re-binning every 2nd interval, 70,000 packets so every attempt
    is split): the chained stage 1 and first attempt
    (defaults), the chained stage 1 alone (SWRT_ODE23_CHAIN_FIRST=0), no
    chain at all (SWRT_ODE23_CHAIN=0) and the launches with event markers
    and event waits (SWRT_ODE23_MARKERS=1) write the same packet_x /
    packet_k / packet_time / pv files, byte for byte."""
    import swraytracing_amd as sw
    from swraytracing_amd import _lib as L
    out = {}
    for name, env in (("first", {}), ("stage1", {"SWRT_ODE23_CHAIN_FIRST": "0"}), ("off", {"SWRT_ODE23_CHAIN": "0"}),
                      ("markers", {"SWRT_ODE23_MARKERS": "1"})):
        for k_, v in (("SWRT_ODE23_CHAIN_FIRST", None), ("SWRT_ODE23_CHAIN", None), ("SWRT_ODE23_MARKERS", None)):
            monkeypatch.delenv(k_, raising=False)
        for k_, v in env.items():
            monkeypatch.setenv(k_, v)
        c = sw.Context(0)
        try:
            d = tmp_path / name
            sw.qg2layersw_raytrace(128, 70_000, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(d), max_steps=48, seed=9,
                                   integrator="ode23", ctx=c)
            out[name] = ({n: (d / n).read_bytes() for n in ("packet_x.bin", "packet_k.bin", "packet_time.bin",
                                                              "pv.bin")},
                         c.debug_get(L.DEBUG_ODE23_CHAINED), c.debug_get(L.DEBUG_ODE23_FIRST_CHAINED))
        finally:
            c.close()
    files, chained, first = out["first"]
    assert chained >= 30 and first >= 30, (chained, first)
    assert out["stage1"][1] >= 30 and out["stage1"][2] == 0
    assert out["off"][1] == 0 and out["off"][2] == 0
    assert out["markers"][1] >= 30 and out["markers"][2] >= 30
    for name in ("stage1", "off", "markers"):
        for fn, b in files.items():
            assert len(b) > 0 and out[name][0][fn] == b, (name, fn)
