"""GPU parity of the device QG PDE stepper (swrt_qg_*, swraytracing_amd/qg.py)
against the oracle (QG1Oracle / QG2Oracle, pinned by tests/test_oracle_qg.py).

Tolerance: the GPU FFT rounds differently from numpy's pocketfft, so every
spectral quantity is compared relative to its max-abs at QG_RTOL.  Over 10-20
PDE steps the nonlinearity does not amplify round-off beyond that (the flows
are smooth, CFL-limited, and the comparison horizon short).  Packets driven by
the device PDE are compared with the oracle pipeline at TRAJ_ATOL.
"""
import numpy as np
import pytest

import swraytracing_amd as sw
from oracle import swrt_oracle as orc

pytestmark = pytest.mark.gpu

QG_RTOL = 1e-11
TRAJ_ATOL = 1e-9


def _rel(a, b):
    return np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(b).max(), 1e-300)


def _one_layer_case(nx=64, seed=146):
    rng = np.random.default_rng(seed)
    q = orc.initial_q(nx, 2 * np.pi, 0.2, 3.0, 5, 8, rng)
    return orc.g2k(q)


def _two_layer_case(nx=64, seed=5):
    rng = np.random.default_rng(seed)
    # qg2layersw_raytrace.m:261-262 uses 10 < |k| <= 30 at production resolution;
    # on these small test grids a lower ring keeps the field resolved
    q1 = orc.initial_q(nx, 20.0, 0.2, 3.0, 1, 3, rng)
    return np.stack([orc.g2k(q1), orc.g2k(-q1)], axis=2)


def test_qg1_steps_match_oracle(ctx):
    """AB3 + filter + inertial-ring forcing.  r_drag = 0 here: update's
    `+ r_drag*K2` term (qgsw_raytrace.m:285, reproduced as written) forces
    every mode by 0.1*K2 and the run blows up within a few steps (both the
    device and the oracle, identically); it is covered separately below."""
    nx, f, Cg = 64, 3.0, 1.0
    qk0 = _one_layer_case(nx)
    m = sw.QGModel.one_layer(qk0, nx, f, Cg, r_drag=0.0, ctx=ctx)
    o = orc.QG1Oracle(qk0, nx, f / Cg, r_drag=0.0, force_strength=0.1, f=f, Cg=Cg, use_filter=True)
    dt = 0.05 * (2 * np.pi / nx) / 0.2
    for n in range(12):
        m.step(dt)
        o.step(dt)
    qk, t, steps = ctx.qg_get()
    assert steps == 12 and abs(t - o.t) < 1e-15
    assert _rel(qk[:, :, 0], o.qk) < QG_RTOL


def test_qg1_r_drag_term_as_written(ctx):
    """The reference's `+ r_drag*K2` (qgsw_raytrace.m:285) on a zero field:
    one Euler step gives qk = dt*0.1*K2 (filtered), exactly as the oracle."""
    nx, f, Cg = 32, 3.0, 1.0
    kmax = nx // 2 - 1
    qk0 = np.zeros((2 * kmax + 1, kmax + 1), complex)
    m = sw.QGModel.one_layer(qk0, nx, f, Cg, r_drag=0.1, force_strength=0.0, ctx=ctx)
    o = orc.QG1Oracle(qk0, nx, f / Cg, r_drag=0.1, force_strength=0.0, f=f, Cg=Cg, use_filter=True)
    m.step(0.01)
    o.step(0.01)
    assert _rel(m.qk[:, :, 0], o.qk) < 1e-14


def test_qg1_filter_off_and_forcing_off(ctx):
    nx, f, Cg = 32, 3.0, 1.0
    qk0 = _one_layer_case(nx, seed=9)
    m = sw.QGModel.one_layer(qk0, nx, f, Cg, r_drag=0.0, force_strength=0.0, use_filter=False, ctx=ctx)
    o = orc.QG1Oracle(qk0, nx, f / Cg, r_drag=0.0, force_strength=0.0, f=f, Cg=Cg, use_filter=False)
    for _ in range(8):
        m.step(0.03)
        o.step(0.03)
    assert _rel(m.qk[:, :, 0], o.qk) < QG_RTOL


def test_qg2_fixed_dt_matches_oracle(ctx):
    nx, L = 64, 20.0
    qk0 = _two_layer_case(nx)
    m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=L, ctx=ctx)
    o = orc.QG2Oracle(qk0, nx, L, 3.0, shear_strength=0.5)
    dt = o.dt
    for _ in range(10):
        m.step(dt)
        o.step(dt)
    assert _rel(m.qk, o.qk) < QG_RTOL


def test_qg2_single_mode_exponential(ctx):
    """J = 0 for one wavevector: the device expLdt alone moves qk; compare
    with the oracle's pageeig exponential (itself checked against expm)."""
    nx, L = 32, 20.0
    kmax = nx // 2 - 1
    qk0 = np.zeros((2 * kmax + 1, kmax + 1, 2), complex)
    qk0[5 + kmax, 2, :] = [0.3 - 0.1j, 0.2 + 0.4j]
    m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=L, ctx=ctx)
    o = orc.QG2Oracle(qk0, nx, L, 3.0, shear_strength=0.5)
    for dt in (0.04, 0.04, 0.07, 0.07, 0.07):  # dt change re-computes the exponentials
        m.step(dt)
        o.step(dt)
    np.testing.assert_allclose(m.qk, o.qk, rtol=1e-12, atol=1e-15)


def test_qg2_adaptive_cfl_sequence(ctx):
    """The driver's CFL rule (qg2layersw_raytrace.m:156-165) on device speeds:
    same dt sequence and state as the oracle."""
    nx, L = 64, 20.0
    qk0 = _two_layer_case(nx, seed=11)
    m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=L, ctx=ctx)
    o = orc.QG2Oracle(qk0, nx, L, 3.0, shear_strength=0.5)
    U0 = m.max_speed()
    assert abs(U0 - o.U0) < 1e-13 * o.U0
    dt = 0.25 * (L / nx) / U0
    assert abs(dt - o.dt) < 1e-13 * o.dt
    # start from a deliberately too-large dt so the rule fires
    o.dt = dt = 3 * dt
    o.exps(o.dt)
    for _ in range(6):
        dt, U0, _ = m.cfl_update(dt, 0.25)
        m.step(dt)
        o.step()
        assert abs(dt - o.dt) <= 1e-12 * o.dt
    assert _rel(m.qk, o.qk) < QG_RTOL


def test_qg_max_speed_async_matches_sync(ctx):
    nx = 64
    m = sw.QGModel.two_layer(_two_layer_case(nx), nx, 3.0, 1.0, ctx=ctx)
    m.step(0.01)
    u_sync = m.max_speed()
    m.max_speed_async()
    ctx.packets_set(np.zeros((4, 2)), np.ones((4, 2)))  # unrelated work queued behind it
    assert m.max_speed_result() == u_sync
    with pytest.raises(sw.SwrtError):
        m.max_speed_result()  # nothing pending


def test_qg_speculative_readback_popped_then_rejected(fresh_ctx):
    """A speculative step whose CFL read-back the caller pops before rejecting
    it (spec -> result -> result -> resolve(0) -> max_speed): the read-back
    FIFO stays consistent, max_speed returns the committed qk's U0 and nothing
    is left pending; the popped speculative U0 is the U0 of the same step taken
    for real (qg2layersw_raytrace.m:152-165: the CFL rule on that step's speed)."""
    nx, dt = 64, 0.01
    m = sw.QGModel.two_layer(_two_layer_case(nx), nx, 3.0, 1.0, ctx=fresh_ctx)
    m.step(dt)
    u_committed = m.max_speed()
    m.max_speed_async()
    m.step_speculative(dt)
    assert m.max_speed_result() == u_committed
    u_spec = m.max_speed_result()
    m.resolve(False)
    assert m.max_speed() == u_committed
    with pytest.raises(sw.SwrtError):
        m.max_speed_result()  # nothing pending
    m.step(dt)
    assert m.max_speed() == u_spec
    # a model call made while a speculative step is pending settles it first
    m.step_speculative(dt)
    m.snapshot(0, which=0, layer=0, ny_period=2 * nx)
    assert not m.spec_pending and m.steps == 2


def test_qg_speculative_snapshot_is_the_accepted_snapshot(fresh_ctx):
    """swrt_qg_snapshot_speculative packs layer 0's grid_U of the pending
    speculative step (qg2layersw_raytrace.m:187-188) before the CFL rule has
    decided: bit for bit the snapshot taken after accepting the step, and
    refused (SWRT_ERR_STATE) without a pending step."""
    nx, dt = 64, 0.01
    ny = 2 * nx
    m = sw.QGModel.two_layer(_two_layer_case(nx), nx, 3.0, 1.0, ctx=fresh_ctx)
    m.step(dt)
    m.max_speed()
    with pytest.raises(sw.SwrtError, match="SWRT_ERR_STATE"):
        m.snapshot_speculative(2, ny_period=ny)
    m.step_speculative(dt)
    m.snapshot_speculative(2, ny_period=ny)
    m.resolve(True)
    m.snapshot(3, which=0, layer=0, ny_period=ny)
    a, b = fresh_ctx.get_field_grid(2, nx), fresh_ctx.get_field_grid(3, nx)
    assert np.ascontiguousarray(a).tobytes() == np.ascontiguousarray(b).tobytes()
    m.max_speed_result()  # the accepted step's read-back


def test_qg_get_q_is_k2g(ctx):
    nx = 64
    qk0 = _two_layer_case(nx)
    m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, ctx=ctx)
    q = m.q()
    for l in range(2):
        assert _rel(q[:, :, l], orc.k2g(qk0[:, :, l])) < 1e-13


@pytest.mark.parametrize("which", [0, 1])
def test_qg_snapshot_is_grid_U(ctx, which):
    """swrt_qg_snapshot == swrt_set_field_qk of the same qk (same device code,
    bit for bit) and == the oracle grid_U (layer 1, u + shear) to FFT round-off."""
    nx, L = 64, 20.0
    qk0 = _two_layer_case(nx)
    m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=L, ctx=ctx)
    m.step(0.01)
    src = (m.qk if which == 0 else None)
    m.snapshot(0, which=which, layer=0, ny_period=2 * nx)
    got = ctx.get_field_grid(0, nx)
    if which == 1:
        src = qk0  # previous qk of the first step is the initial state
    ctx.set_field_qk(1, src[:, :, 0], nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
    ref = ctx.get_field_grid(1, nx)
    np.testing.assert_array_equal(got, ref)
    kx_, ky_, K2 = orc.wavenumber_grids(nx, L, scale=True)
    flow = orc.grid_U(src[:, :, 0], 3.0, K2, kx_, ky_, 0.5)
    for i, name in enumerate(orc.FIELD_ORDER):
        assert _rel(got[i], np.asarray(flow[name]).ravel(order="F")) < 1e-12


@pytest.mark.parametrize("nx", [16, 64])
def test_qk_snapshot_ghost_records(ctx, nx):
    """pack_pairs_kernel writes the periodic ghost records itself: the node
    array of swrt_set_field_qk evaluates, at points in every edge and corner
    cell, bit for bit like the same planes packed by swrt_set_field_grid."""
    L = 20.0
    rng = np.random.default_rng(4)
    qk = _two_layer_case(nx)[:, :, 0]
    ctx.set_field_qk(0, qk, nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
    ctx.set_field_grid(1, ctx.get_field_grid(0, nx), nx, L, 2 * nx)
    dx = L / nx
    edge = np.concatenate([np.arange(-3, 4) * dx, L / 2 + np.arange(-4, 4) * dx, -L / 2 + np.arange(-4, 4) * dx])
    X, Y = np.meshgrid(edge, edge)
    x = np.concatenate([X.ravel(), rng.uniform(-L, L, 2000)]) + 1e-3 * dx
    y = np.concatenate([Y.ravel(), rng.uniform(-2 * L, 2 * L, 2000)]) - 2e-3 * dx
    a = ctx.eval(x, y, nslots=1, bump=orc.BUMP_QG)
    ctx.swap_slots(0, 1)
    b = ctx.eval(x, y, nslots=1, bump=orc.BUMP_QG)
    np.testing.assert_array_equal(a, b)


def test_swap_slots(ctx):
    nx = 32
    a = np.random.default_rng(1).random((6, nx * nx))
    b = np.random.default_rng(2).random((6, nx * nx))
    ctx.set_field_grid(0, a, nx, 2 * np.pi)
    ctx.set_field_grid(1, b, nx, 2 * np.pi)
    ctx.swap_slots(0, 1)
    np.testing.assert_array_equal(ctx.get_field_grid(0, nx), b)
    np.testing.assert_array_equal(ctx.get_field_grid(1, nx), a)


def test_qgsw_driver_packets_match_oracle_pipeline(ctx, oracle_lib, tmp_path):
    """qgsw_raytrace on the device (PDE + snapshots + fused packets) against
    the same pipeline on the CPU oracle: QG1Oracle steps, grid_U of (prev_qk,
    qk), the C-oracle leapfrog with the blend; 12 PDE steps, all packet-active."""
    nx, N, nsub = 64, 300, 3
    f, Cg = 3.0, 1.0
    res = sw.qgsw_raytrace(nx, N, 4.0, 10.0, 0.0, 0.2, f, Cg, out_dir=str(tmp_path), nsub=nsub,
                           max_steps=12, seed=146, r_drag=0.0, ctx=ctx)
    assert res["steps"] == 12
    xg = sw.read_field(str(tmp_path / "packet_x"), N, 2, 1)
    kg = sw.read_field(str(tmp_path / "packet_k"), N, 2, 1)
    tg = sw.read_field(str(tmp_path / "packet_time"))
    frames = 1 + 12 // 5
    assert xg.shape == (N, 2, frames) and tg.shape == (1, frames)
    _load_data_reads(tmp_path, nx, N, f, Cg, 0.2)
    # oracle pipeline from the same initial state
    rng = np.random.default_rng(146)
    L = 2 * np.pi
    q = sw.qg.initial_q(nx, L, 0.2, f / Cg, 5, 8, rng)
    x, k = sw.qg._packets(N, L, 4.0, f, Cg, rng)
    o = orc.QG1Oracle(orc.g2k(q), nx, f / Cg, r_drag=0.0, f=f, Cg=Cg)
    dt = res["dt"]
    kx_, ky_, K2 = orc.wavenumber_grids(nx)
    from tests.test_gpu_parity import _planes
    for step in range(1, 13):
        prev = o.qk.copy()
        o.step(dt)
        p0 = _planes(orc.grid_U(prev, f / Cg, K2, kx_, ky_))
        p1 = _planes(orc.grid_U(o.qk, f / Cg, K2, kx_, ky_))
        x, k, _, _ = oracle_lib.leapfrog(p0, p1, 0.5 / nsub, 1.0 / nsub, nx, nx, L / nx, orc.BUMP_QG, x, k,
                                         dt / nsub, nsub, f, Cg ** 2)
    xw = np.mod(x + L / 2, L) - L / 2
    xs, ks = ctx.packets_get()
    np.testing.assert_allclose(xs, x, atol=TRAJ_ATOL, rtol=0)
    np.testing.assert_allclose(ks, k, atol=TRAJ_ATOL, rtol=0)
    assert np.abs(xg[:, :, -1]).max() <= L / 2 + 1e-12
    assert np.isfinite(xw).all()


def test_qg2layer_driver_runs_and_writes(ctx, tmp_path):
    nx, N = 64, 500
    res = sw.qg2layersw_raytrace(nx, N, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(tmp_path), nsub=2,
                                 max_steps=30, seed=5, ctx=ctx)
    assert res["steps"] == 30
    xg = sw.read_field(str(tmp_path / "packet_x"), N, 2, 1)
    assert xg.shape[-1] == 1 + 30 // 25
    assert np.isfinite(xg).all()
    pv = sw.read_field(str(tmp_path / "pv"), nx, nx, 2)
    assert pv.shape == (nx, nx, 2)
    _load_data_reads(tmp_path, nx, N, 3.0, 1.0, 0.2)


def _load_data_reads(d, nx, N, f, Cg, Ug):
    """analysis/load_data.m:18-32 on a driver's output directory, unchanged:
    the five textscan calls on run.log (header offsets 10 and 7), then
    read_field(packet_time) and read_field(packet_x/k, Npackets, 2, 1, 1:frames)."""
    from tests.matlab_textscan import load_data_header
    h = load_data_header(str(d / "run.log"))
    assert h["resolution"] == (nx, nx) and h["Npackets"] == N
    assert h["f"] == f and h["Cg"] == Cg and h["Ug"][0] == Ug and h["Ug"][1] > 0
    t = sw.read_field(str(d / "packet_time"))
    frames = t.shape[1]
    for name in ("packet_x", "packet_k"):
        a = sw.read_field(str(d / name), h["Npackets"], 2, 1, list(range(1, frames + 1)))
        a = a.reshape(N, 2, frames)
        assert np.isfinite(a).all()
    assert open(d / "run.log").read().rstrip("\n").split("\n")[-1].startswith("Real time elapsed: ")


def test_qg2_driver_packet_streams_identical_files(tmp_path):
    """The 2-layer driver (QG stream renaming snapshot slots beside the packet
    launches) with the packet launches split over two streams writes the
    same packet files, byte for byte, as with one."""
    import swraytracing_amd as sw
    files = {}
    for streams in (1, 2):
        c = sw.Context(0)
        try:
            c.set_packet_streams(streams)
            d = tmp_path / f"s{streams}"
            # >= 65,536 packets: smaller ensembles always take one stream
            sw.qg2layersw_raytrace(128, 70_000, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(d), nsub=5, max_steps=60,
                                   seed=5, ctx=c)
            files[streams] = {n: (d / f"{n}.bin").read_bytes() for n in ("packet_x", "packet_k", "packet_time")}
        finally:
            c.close()
    assert files[1] == files[2]
    assert len(files[1]["packet_x"]) == 8 * 70_000 * 2 * (1 + 60 // 25)


def test_golden_qg_fixture(ctx):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_qg.npz"))
    nx = int(g["nx"])
    m1 = sw.QGModel.one_layer(g["qk1_0"], nx, 3.0, 1.0, r_drag=0.0, ctx=ctx)
    m1.step(float(g["dt1"]), 8)
    assert _rel(m1.qk[:, :, 0], g["qk1_8"]) < QG_RTOL
    m2 = sw.QGModel.two_layer(g["qk2_0"], nx, 3.0, 1.0, L=float(g["L2"]), ctx=ctx)
    dt = 0.25 * (float(g["L2"]) / nx) / m2.max_speed()
    for want in g["dts2"]:
        dt, _, _ = m2.cfl_update(dt, 0.25)
        assert abs(dt - want) <= 1e-12 * want
        m2.step(dt)
    assert _rel(m2.qk, g["qk2_8"]) < QG_RTOL


def _driver_files(ctx, d, layers, separate, fused, intervals):
    ctx.qg_set_stream(separate)
    ctx.qg_set_fused(fused)
    d.mkdir()
    if layers == 2:
        sw.qg2layersw_raytrace(128, 200_000, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(d), nsub=2, max_steps=30,
                               seed=5, packet_intervals=intervals, ctx=ctx)
    else:
        sw.qgsw_raytrace(64, 50_000, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(d), nsub=2, max_steps=12,
                         seed=146, r_drag=0.0, packet_intervals=intervals, ctx=ctx)
    return [open(d / name, "rb").read() for name in ("packet_x.bin", "packet_k.bin", "pv.bin", "packet_time.bin")]


@pytest.mark.parametrize("layers", [1, 2])
def test_qg_stream_overlap_and_fusion_bit_identical(ctx, tmp_path, layers):
    """The QG PDE on its own stream with snapshot renaming
    (swrt_qg_set_stream), the fused post-step transforms (swrt_qg_set_fused)
    and packet intervals grouped 4 per call (PDE run ahead,
    swrt_advance_intervals) — all defaults — give the same packets, frames,
    PV and frame times (the CFL dt sequence) as one stream without fusion,
    one interval per call.  The 2-layer case has packet launches long enough
    that snapshots meet in-flight reads; frames every 5 (1-layer) and 25
    (2-layer) steps cut groups short."""
    try:
        ref = _driver_files(ctx, tmp_path / "plain", layers, False, False, 1)
        for sep, fused, iv in [(True, True, 4), (True, False, 1), (False, True, 4), (True, True, 3)]:
            got = _driver_files(ctx, tmp_path / f"s{int(sep)}f{int(fused)}i{iv}", layers, sep, fused, iv)
            assert all(len(u) > 0 and u == v for u, v in zip(got, ref)), (sep, fused, iv)
    finally:
        ctx.qg_set_stream(True)
        ctx.qg_set_fused(True)


@pytest.mark.parametrize("nx", [64, 512, 1024, 2048])
def test_qg_fused_speed_and_snapshot_match_unfused(ctx, nx):
    """U0 and the layer-0 snapshot of the current qk from the post-step
    transforms equal the separate calls' bit for bit (2 layers, AB3 steps).
    The sizes cover every post-step shape: spectra fused into the row pass
    (<= 512), the Jacobian fused into the forward row pass (<= 1024), the
    one-buffer FFT (<= 1024) and the ping-pong FFT (2048)."""
    out = {}
    try:
        # fused with the speed first (both post-step phases, then the pack) and
        # with the snapshot first (the inverse phase alone, the Jacobian phase
        # on the speed request that follows)
        for mode in ("unfused", "fused", "fused-snapshot-first"):
            ctx.qg_set_fused(mode != "unfused")
            m = sw.QGModel.two_layer(_two_layer_case(nx, seed=11), nx, 3.0, 1.0, L=20.0, ctx=ctx)
            dt = 0.25 * (20.0 / nx) / m.max_speed()
            for _ in range(4):
                m.step(dt)
            if mode == "fused-snapshot-first":
                m.snapshot(0, which=0, ny_period=2 * nx)
                U0 = m.max_speed()
            else:
                U0 = m.max_speed()
                m.snapshot(0, which=0, ny_period=2 * nx)
            m.step(dt)
            m.snapshot(1, which=0, ny_period=2 * nx)
            out[mode] = (U0, m.max_speed(), ctx.get_field_grid(0, nx), ctx.get_field_grid(1, nx), m.qk)
    finally:
        ctx.qg_set_fused(True)
    a = out["unfused"]
    for mode in ("fused", "fused-snapshot-first"):
        b = out[mode]
        assert a[0] == b[0] and a[1] == b[1]
        for u, v in zip(a[2:], b[2:]):
            assert np.array_equal(np.ascontiguousarray(u).view(np.uint64), np.ascontiguousarray(v).view(np.uint64))


@pytest.mark.parametrize("nx", [64, 512])
def test_qg_transform_grouping_bit_identical(nx):
    """The post-step transforms take one vector per workgroup while a context
    with packets runs its QG calls on the separate stream (the driver loop),
    two otherwise (swrt_api.hip fft_group): the same per-vector FFTs, so U0,
    the snapshots and qk agree bit for bit between a context without and one
    with packets."""
    out = []
    for with_packets in (False, True):
        c = sw.Context(0)
        try:
            if with_packets:
                rng = np.random.default_rng(3)
                c.packets_set(20.0 * rng.random((1000, 2)) - 10.0, rng.normal(0.0, 3.0, (1000, 2)))
            m = sw.QGModel.two_layer(_two_layer_case(nx, seed=11), nx, 3.0, 1.0, L=20.0, ctx=c)
            dt = 0.25 * (20.0 / nx) / m.max_speed()
            for _ in range(4):
                m.step(dt)
            U0 = m.max_speed()
            m.snapshot(0, which=0, ny_period=2 * nx)
            out.append((U0, c.get_field_grid(0, nx).copy(), m.qk))
        finally:
            c.close()
    (u_a, f_a, q_a), (u_b, f_b, q_b) = out
    assert u_a == u_b
    assert np.array_equal(f_a.view(np.uint64), f_b.view(np.uint64))
    assert np.array_equal(np.ascontiguousarray(q_a).view(np.uint64), np.ascontiguousarray(q_b).view(np.uint64))


def _ring_qk(nx, L, rng, Ug=0.2, kmin=10, kmax_ring=30):
    """Production-size 2-layer state (q1, -q1) on the driver's 10 < |k| <= 30
    ring (qg2layersw_raytrace.m:261-262) with random phases, scaled to
    max|U| = Ug of layer 1 — built in the spectrum directly (initial_q's
    grid loop is minutes of numpy at 512^2)."""
    kmax = nx // 2 - 1
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(kmax + 1)[None, :]
    r2 = kx * kx + ky * ky
    qk = np.where((r2 > kmin ** 2) & (r2 <= kmax_ring ** 2),
                  np.exp(2j * np.pi * rng.random((2 * kmax + 1, kmax + 1))), 0)
    kx_, ky_, K2 = orc.wavenumber_grids(nx, L, scale=True)
    fl = orc.grid_U(qk, 3.0, K2, kx_, ky_)
    qk = qk * (Ug / np.sqrt((fl["u"] ** 2 + fl["v"] ** 2).max()))
    return np.stack([qk, -qk], axis=2)


def test_qg2_driver_loop_512_matches_oracle_pipeline(ctx, oracle_lib):
    """The benched configuration end to end: 512^2 x 2 layers, 1e6 packets,
    the driver's own loop body (TwoLayerLoop: adaptive CFL, PDE on the QG
    stream with the fused post-step transforms, snapshots renamed past
    in-flight packet reads, 5 leapfrog substeps per interval) for 6 PDE steps
    against QG2Oracle + the oracle's grid_U + the C-oracle leapfrog on a
    random subset of 3000 packets.  Same dt sequence, qk within QG_RTOL,
    the last snapshot within the field tolerance, packets within TRAJ_ATOL."""
    nx, L, f, Cg, N, nsub, nsteps = 512, 20.0, 3.0, 1.0, 1_000_000, 5, 6
    rng = np.random.default_rng(512)
    qk0 = _ring_qk(nx, L, rng)
    x, k = sw.qg._packets(N, L, 4.0, f, Cg, rng)
    model = sw.QGModel.two_layer(qk0, nx, f, Cg, L=L, ctx=ctx)
    ens = sw.PacketEnsemble(x, k, L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * np.pi / L, nlayers=2,
                            bump=sw.BUMP_QG, ctx=ctx)
    U0 = model.max_speed()
    loop = sw.TwoLayerLoop(model, ens, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=nsub)
    for _ in range(nsteps):
        assert loop.step()
    loop.flush()
    xs, ks = ens.state()
    snap = ctx.get_field_grid(0, nx)  # grid_U of the last qk (slot 0 after the swap)
    qk_dev = model.qk

    o = orc.QG2Oracle(qk0, nx, L, f / Cg, shear_strength=0.5)
    kx_, ky_, K2 = orc.wavenumber_grids(nx, L, scale=True)
    idx = np.sort(rng.choice(N, 3000, replace=False))
    xo, ko = x[idx], k[idx]
    from tests.test_gpu_parity import _planes
    flow = None
    for s in range(nsteps):
        prev = o.qk[:, :, 0].copy()
        o.step()
        assert abs(loop.dts[s] - o.dt) <= 1e-12 * o.dt, (s, loop.dts[s], o.dt)
        p0 = _planes(orc.grid_U(prev, f / Cg, K2, kx_, ky_, 0.5))
        flow = orc.grid_U(o.qk[:, :, 0], f / Cg, K2, kx_, ky_, 0.5)
        xo, ko, _, _ = oracle_lib.leapfrog(p0, _planes(flow), 0.5 / nsub, 1.0 / nsub, nx, 2 * nx, L / nx,
                                           orc.BUMP_QG, xo, ko, o.dt / nsub, nsub, f, Cg ** 2)
    assert _rel(qk_dev, o.qk) < QG_RTOL
    for i, name in enumerate(orc.FIELD_ORDER):
        assert _rel(snap[i], np.asarray(flow[name]).ravel(order="F")) < 1e-12, name
    np.testing.assert_allclose(xs[idx], xo, atol=TRAJ_ATOL, rtol=0)
    np.testing.assert_allclose(ks[idx], ko, atol=TRAJ_ATOL, rtol=0)
    assert np.isfinite(xs).all() and np.isfinite(ks).all()


def test_qg2_512_adaptive_cfl_matches_oracle(ctx):
    """The 2-layer PDE alone at 512^2 with a dt large enough that the CFL rule
    fires: same dt sequence and qk as QG2Oracle (fused transforms + QG stream,
    the defaults), and U0 of the device equal to the oracle's."""
    nx, L = 512, 20.0
    qk0 = _ring_qk(nx, L, np.random.default_rng(7), Ug=0.3)
    m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=L, ctx=ctx)
    o = orc.QG2Oracle(qk0, nx, L, 3.0, shear_strength=0.5)
    U0 = m.max_speed()
    assert abs(U0 - o.U0) < 1e-12 * o.U0
    o.dt = dt = 2.5 * o.dt
    o.exps(o.dt)
    fired = 0
    for _ in range(5):
        dt, U0, changed = m.cfl_update(dt, 0.25)
        fired += changed
        m.step(dt)
        o.step()
        assert abs(dt - o.dt) <= 1e-12 * o.dt
    assert fired >= 1
    assert _rel(m.qk, o.qk) < QG_RTOL


def test_integrator_substitution_preserves_omega_statistics(ctx, tmp_path):
    """The drivers replace the reference's ode23 packet integrator
    (qg2layersw_raytrace.m:195) by nsub fused leapfrog substeps per PDE
    interval.  Here the 2-layer driver runs 1600 PDE steps at 128^2 with
    20,000 packets twice from the same PDE state and packets — once with each
    integrator (the PDE does not see the packets, so both runs see the same
    flow) — and the science output of analysis/load_data.m:33-52,63 is
    compared: omega = sqrt(f^2 + Cg^2 |k|^2) per packet and frame.
      * the per-packet difference grows along the run (ode23's local error
        control at RelTol 1e-3 vs the symplectic substeps), so the comparison
        is statistical;
      * mean omega(t)/f of every frame agrees within 4 standard errors;
      * the omega distributions of the last frames agree by a two-sample KS
        test at alpha = 0.001 (D <= 1.95 sqrt(2/N));
      * the load_data.m energy spectrum (center .* histcounts(omega, edges),
        300 bins) carries the same total to within 4 standard errors."""
    from scipy import stats
    nx, N, f, Cg = 128, 20_000, 3.0, 1.0
    om = {}
    for integ in ("leapfrog", "ode23"):
        d = tmp_path / integ
        res = sw.qg2layersw_raytrace(nx, N, 4.0, 1e5, 0.0, 0.2, f, Cg, out_dir=str(d), nsub=5, max_steps=1600,
                                     seed=11, integrator=integ, ctx=ctx)
        assert res["steps"] == 1600
        k = sw.read_field(str(d / "packet_k"), N, 2, 1)  # N x 2 x frames
        om[integ] = np.sqrt(f * f + Cg * Cg * (k ** 2).sum(axis=1))  # load_data.m:33, N x frames
    a, b = om["leapfrog"], om["ode23"]
    assert a.shape == b.shape and a.shape[1] == 1 + 1600 // 25
    np.testing.assert_array_equal(a[:, 0], b[:, 0])  # same initial packets
    # the per-packet difference grows, and the distribution evolved from its start (all omega_0 = 4f)
    dif = np.abs(a - b).max(axis=0)
    assert dif[-1] > 4 * dif[2], dif
    assert a[:, -1].std() > 0.01 * f
    for fr in range(a.shape[1]):  # mean_omega = mean(omega)/f (load_data.m:63)
        se = np.sqrt(a[:, fr].var() / N + b[:, fr].var() / N)
        assert abs(a[:, fr].mean() - b[:, fr].mean()) <= 4 * se + 1e-12, fr
    wa, wb = a[:, -4:].ravel(), b[:, -4:].ravel()
    D = stats.ks_2samp(wa, wb).statistic
    assert D <= 1.95 * np.sqrt(2.0 / N), D  # N independent packets per run (frames are correlated)
    edges = np.linspace(0, max(wa.max(), wb.max()), 300)
    center = (edges[1:] + edges[:-1]) / 2
    ea = (center * np.histogram(wa, edges)[0]).sum() / wa.size
    eb = (center * np.histogram(wb, edges)[0]).sum() / wb.size
    assert abs(ea - eb) <= 4 * np.sqrt(wa.var() / N + wb.var() / N) + (edges[1] - edges[0])


def _speculative_driver_run(ctx, speculate, integrator="leapfrog"):
    nx, L, f, Cg, N = 128, 20.0, 3.0, 1.0, 70_000
    rng = np.random.default_rng(21)
    qk0 = _ring_qk(nx, L, rng)
    x, k = sw.qg._packets(N, L, 4.0, f, Cg, rng)
    model = sw.QGModel.two_layer(qk0, nx, f, Cg, L=L, ctx=ctx)
    ens = sw.PacketEnsemble(x, k, L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * np.pi / L, nlayers=2,
                            bump=sw.BUMP_QG, ctx=ctx)
    U0 = model.max_speed()
    loop = sw.TwoLayerLoop(model, ens, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=5, speculate=speculate,
                           integrator=integrator)
    U0s = []
    for s in range(12):
        if s == 6:
            loop.dt = 3.0 * loop.dt  # the CFL rule fires at this step: a queued speculative step is dropped
        assert loop.step()
        U0s.append(loop.U0)
    loop.flush()
    import swraytracing_amd._lib as L_
    chained = ctx.debug_get(L_.DEBUG_ODE23_CHAINED)
    first_chained = ctx.debug_get(L_.DEBUG_ODE23_FIRST_CHAINED)
    qk_pending = model.qk  # the committed step while a speculative one is queued
    loop.settle()
    xs, ks = ens.state()
    return model.qk, qk_pending, xs, ks, list(loop.dts), U0s, model.t, model.steps, chained, first_chained


@pytest.mark.parametrize("integrator", ["leapfrog", "ode23"])
def test_qg2_speculative_steps_bit_identical(fresh_ctx, integrator):
    """TwoLayerLoop(speculate=True) queues each next PDE step with the current
    dt before it reads this step's U0 (swrt_qg_step_speculative), then the CFL
    rule (qg2layersw_raytrace.m:156-165) accepts it or — when dt changes —
    drops it (swrt_qg_resolve) and steps again.  Against the plain loop: the
    same dt sequence (one change forced mid-run), U0 values, qk, PDE time and
    step count, and every packet's bits; swrt_qg_get reports the committed
    step while a speculative one is queued.  With the drivers' ode23 the next
    step is queued from inside the interval (swrt_ode23_run_hooked's hook,
    beside its attempts split over two streams)."""
    runs = {}
    for spec in (False, True):
        runs[spec] = _speculative_driver_run(fresh_ctx, spec, integrator)
    a, b = runs[False], runs[True]
    assert a[4] == b[4] and len(set(a[4])) >= 2  # dts, with a change
    assert a[5] == b[5]  # U0 per step
    for u, v in zip(a[:4], b[:4]):
        assert np.ascontiguousarray(u).tobytes() == np.ascontiguousarray(v).tobytes()
    assert a[6] == b[6] and a[7] == b[7] == 12
    if integrator == "ode23":
        # the speculative loop chains each interval's stage 1 to the previous
        # call (swrt_ode23_chain_next); the forced dt change drops one chain
        # (a fresh snapshot rewrites slot 1) and the plain loop never arms it
        assert a[8] == 0 and 8 <= b[8] <= 10, (a[8], b[8])
        # and the first attempt behind each chained stage 1, but at the dt
        # change (the chain assumed tfinal = the previous dt)
        assert a[9] == 0 and b[8] - 1 <= b[9] <= b[8], (a[9], b[9])


@pytest.mark.parametrize("nx", [64, 512])
def test_qg2_column_jacobian_fusion_bit_identical(fresh_ctx, nx):
    """Two-layer fused mode: the inverse column pass fused with the Jacobian,
    the CFL max and J's first forward pass (fft_cols_jacobian2_kernel, the
    default) against the separate column pass + Jacobian-rows kernel
    (SWRT_DEBUG_QG_JFUSE 0): the same qk after 8 AB3 steps, the same U0 at
    every step and the same packet snapshot, bit for bit
    (qg2layersw_raytrace.m:309-323, grid_U.m)."""
    import swraytracing_amd._lib as L
    ctx = fresh_ctx
    L_ = 20.0
    qk0 = _two_layer_case(nx) if nx == 64 else _ring_qk(nx, L_, np.random.default_rng(9))
    out = {}
    for fuse in (0, 1):
        ctx.debug_set(L.DEBUG_QG_JFUSE, fuse)
        m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=L_, ctx=ctx)
        U = [m.max_speed()]
        dt = 0.25 * (L_ / nx) / U[0]
        for _ in range(8):
            m.step(dt)
            U.append(m.max_speed())
        m.snapshot(0, which=0, layer=0, ny_period=2 * nx)
        out[fuse] = (np.ascontiguousarray(m.qk).tobytes(), U, ctx.get_field_grid(0, nx).tobytes())
    ctx.debug_set(L.DEBUG_QG_JFUSE, 1)
    assert out[0][1] == out[1][1]
    assert out[0][0] == out[1][0]
    assert out[0][2] == out[1][2]


@pytest.mark.parametrize("layers,nx", [(1, 32), (1, 256), (2, 16), (2, 64), (2, 512)])
def test_qg_update_column_fusion_bit_identical(fresh_ctx, layers, nx):
    """Fused mode: the last pass of J's forward transform inside the AB3
    update (qg_update_cols_kernel, the default: each workgroup transforms
    the FFT columns kx = +-r and updates every wavenumber (+-r, ky) from
    LDS, storing only the new tendency and renaming the history buffers)
    against the separate column pass + update (SWRT_DEBUG_QG_UPDATE_COLS 0):
    the same qk and U0 after every step, bit for bit, through the Euler and
    AB2 start steps, AB3 steps, a rejected and an accepted speculative step
    (swrt_qg_resolve's buffer renaming), and steps after them that read the
    renamed history (qgsw_raytrace.m:121-137, qg2layersw_raytrace.m:168-181,
    309-323)."""
    import swraytracing_amd._lib as L
    ctx = fresh_ctx
    out = {}
    try:
        for cols in (0, 1):
            ctx.debug_set(L.DEBUG_QG_UPDATE_COLS, cols)
            if layers == 1:
                # (r_drag as written forces every mode: at 256^2 the run overflows
                # within these steps, and NaN payloads carry no parity)
                m = sw.QGModel.one_layer(_one_layer_case(nx), nx, 3.0, 1.0, r_drag=0.1 if nx < 64 else 0.0, ctx=ctx)
                Lx = 2 * np.pi
            else:
                qk0 = _two_layer_case(nx) if nx < 512 else _ring_qk(nx, 20.0, np.random.default_rng(9))
                m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=20.0, ctx=ctx)
                Lx = 20.0
            U = [m.max_speed()]
            dt = 0.25 * (Lx / nx) / U[0]
            trace = []
            for s in range(9):
                if s == 3:
                    m.step_speculative(dt)
                    m.resolve(False)
                if s == 5:
                    m.step_speculative(dt)
                    m.resolve(True)
                else:
                    m.step(dt)
                U.append(m.max_speed())
                trace.append(np.ascontiguousarray(m.qk).tobytes())
            out[cols] = (U, trace, m.steps)
    finally:
        ctx.debug_set(L.DEBUG_QG_UPDATE_COLS, 1)
    assert out[0][2] == out[1][2] == 9
    assert np.isfinite(out[1][0]).all()
    assert out[0][0] == out[1][0]
    for s, (a, b) in enumerate(zip(out[0][1], out[1][1])):
        assert a == b, s
