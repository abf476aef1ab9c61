"""GPU parity: the HIP path through the C ABI vs the CPU oracle.

Packet kernels (interpolate / eval / leapfrog) are bit-exact: same IEEE fp64
operations in the same order, no FMA contraction, correctly rounded div/sqrt.
Field preparation (g2k / k2g / grid_U / SpectralScheme ctor) uses a different
FFT than numpy, so it is compared within a stated fp64 tolerance:
  FIELD_RTOL = 1e-13 of the field's max-abs (FFT round-off ~ log2(n) eps).
Trajectories built on GPU-prepared fields inherit that round-off; over <= 100
steps they are compared at TRAJ_ATOL = 1e-10 (BASELINE.md parity row).
"""
import math
import os

import numpy as np
import pytest

from oracle import swrt_oracle as orc
from tests.conftest import ROOT, periodic_grid

pytestmark = pytest.mark.gpu

FIELD_RTOL = 1e-13
TRAJ_ATOL = 1e-10
GOLD = os.path.join(ROOT, "tests", "golden")


def _planes(flow):
    return np.ascontiguousarray(np.stack([np.asarray(flow[n]).ravel(order="F") for n in orc.FIELD_ORDER]))


def _edge_points(nx, L, rng, n=4096):
    dx = L / nx
    pts = [0.0, -0.0, -1e-17, 1e-17, L, -L, L / 2, -L / 2, 3 * dx, -5 * dx, 1e3 * L + dx / 3,
           -7e2 * L - 1e-9, np.nextafter(dx, 0), np.nextafter(dx, 1), 1e6, -1e6]
    x = np.concatenate([rng.uniform(-3 * L, 3 * L, n), np.array(pts)])
    y = np.concatenate([rng.uniform(-3 * L, 3 * L, n), np.array(pts[::-1])])
    return x, y


def test_eval_bitexact(ctx, oracle_lib, qg_case):
    c = qg_case
    nx, L = c["nx"], c["L"]
    pl = _planes(c["flow"])
    ctx.set_field_grid(0, pl, nx, L)
    rng = np.random.default_rng(7)
    x, y = _edge_points(nx, L, rng)
    for bump in (orc.BUMP_SW, orc.BUMP_QG):
        g = ctx.eval(x, y, nslots=1, bump=bump)
        o = oracle_lib.eval6(pl, None, 0.0, nx, nx, L / nx, bump, x, y)
        np.testing.assert_array_equal(g, o)
    # numpy oracle agrees too (independent restatement)
    I = orc.interpolate_fields(x[:300], y[:300], c["flow"], L / nx, orc.BUMP_QG)
    np.testing.assert_array_equal(ctx.eval(x[:300], y[:300], bump=orc.BUMP_QG), I)


def test_eval_blend_two_layer_bitexact(ctx, oracle_lib, qg_case):
    c = qg_case
    nx, L = c["nx"], c["L"]
    fl2 = {n: np.asarray(v) * 0.9 + 0.01 for n, v in c["flow"].items()}
    p0, p1 = _planes(c["flow"]), _planes(fl2)
    ctx.set_field_grid(0, p0, nx, L, 2 * nx)
    ctx.set_field_grid(1, p1, nx, L, 2 * nx)
    rng = np.random.default_rng(8)
    x, y = _edge_points(nx, L, rng)
    for alpha in (0.0, 0.37, 1.0):
        g = ctx.eval(x, y, nslots=2, alpha=alpha, bump=orc.BUMP_QG)
        o = oracle_lib.eval6(p0, p1, alpha, nx, 2 * nx, L / nx, orc.BUMP_QG, x, y)
        np.testing.assert_array_equal(g, o)


def test_interpolate_generic_matches_numpy_oracle(ctx):
    nx, L = 48, 20.0  # non-power-of-two grid, qg2layer domain length
    X, Y = periodic_grid(nx, L)
    F = np.zeros((nx, nx, 2))
    F[:, :, 0] = np.sin(2 * np.pi * X / L) * np.cos(4 * np.pi * Y / L)
    F[:, :, 1] = -3.0
    rng = np.random.default_rng(9)
    x, y = _edge_points(nx, L, rng, 2000)
    for FF in (F, F[:, :, 0]):
        g = ctx.interpolate(x, y, FF, L / nx, L / nx, orc.BUMP_QG)
        o = orc.interpolate(x, y, FF, L / nx, L / nx, orc.BUMP_QG)
        np.testing.assert_array_equal(g, o)


def test_leapfrog_bitexact_steady_with_history(ctx, oracle_lib, qg_case):
    c = qg_case
    nx, L = c["nx"], c["L"]
    pl = _planes(c["flow"])
    ctx.set_field_grid(0, pl, nx, L)
    nsteps = 150  # > one launch (64 steps): exercises the chunked launch path
    xg, kg, hxg, hkg = ctx.leapfrog(c["x"], c["k"], c["dt"], nsteps, c["f"], 1.0, bump=orc.BUMP_SW,
                                    save_every=10)
    xo, ko, hxo, hko = oracle_lib.leapfrog(pl, None, 0, 0, nx, nx, L / nx, orc.BUMP_SW, c["x"], c["k"],
                                           c["dt"], nsteps, c["f"], 1.0, save_every=10)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)
    np.testing.assert_array_equal(hxg, hxo)
    np.testing.assert_array_equal(hkg, hko)


def test_history_capacity_follows_the_packet_count(ctx, oracle_lib, qg_case):
    """A small ensemble with many frames, then a 64x larger one with few: the
    history capacity is counted in doubles (frames x 2 x n), so the second
    call grows the buffers (a capacity counted in frames let it write past
    them — found through a test order that ran the interval tests after
    these)."""
    c = qg_case
    nx, L = c["nx"], c["L"]
    pl = _planes(c["flow"])
    ctx.set_field_grid(0, pl, nx, L)
    xs, ks = c["x"][:16], c["k"][:16]
    ctx.leapfrog(xs, ks, c["dt"], 64, c["f"], 1.0, bump=orc.BUMP_SW, save_every=1)
    rng = np.random.default_rng(3)
    xb = np.concatenate([c["x"] + rng.normal(0, 1e-3, c["x"].shape) for _ in range(4)])
    kb = np.concatenate([c["k"]] * 4)
    xg, kg, hxg, hkg = ctx.leapfrog(xb, kb, c["dt"], 8, c["f"], 1.0, bump=orc.BUMP_SW, save_every=4)
    xo, ko, hxo, hko = oracle_lib.leapfrog(pl, None, 0, 0, nx, nx, L / nx, orc.BUMP_SW, xb, kb, c["dt"], 8,
                                           c["f"], 1.0, save_every=4)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(hxg, hxo)
    np.testing.assert_array_equal(hkg, hko)


def test_leapfrog_blend_bitexact(ctx, oracle_lib, qg_case):
    c = qg_case
    nx, L = c["nx"], c["L"]
    fl2 = {n: np.asarray(v) * 1.1 for n, v in c["flow"].items()}
    p0, p1 = _planes(c["flow"]), _planes(fl2)
    ctx.set_field_grid(0, p0, nx, L, 2 * nx)
    ctx.set_field_grid(1, p1, nx, L, 2 * nx)
    nsub = 8
    xg, kg, _, _ = ctx.leapfrog(c["x"], c["k"], c["dt"] / nsub, nsub, c["f"], 1.0, nslots=2,
                                alpha0=0.5 / nsub, dalpha=1.0 / nsub, bump=orc.BUMP_QG)
    xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.5 / nsub, 1.0 / nsub, nx, 2 * nx, L / nx, orc.BUMP_QG,
                                       c["x"], c["k"], c["dt"] / nsub, nsub, c["f"], 1.0)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)


def test_golden_fixtures_bitexact(ctx):
    g = np.load(os.path.join(GOLD, "golden_steady.npz"))
    nx = int(g["nx"])
    ctx.set_field_grid(0, g["planes"], nx, float(g["L"]))
    x, k, hx, hk = ctx.leapfrog(g["x0"], g["k0"], float(g["dt"]), int(g["nsteps"]), float(g["f"]),
                                float(g["gH"]), bump=float(g["bump"]), save_every=int(g["save_every"]))
    np.testing.assert_array_equal(x, g["x"])
    np.testing.assert_array_equal(k, g["k"])
    np.testing.assert_array_equal(hx, g["hist_x"].transpose(0, 2, 1))
    np.testing.assert_array_equal(hk, g["hist_k"].transpose(0, 2, 1))
    b = np.load(os.path.join(GOLD, "golden_blend.npz"))
    nx = int(b["nx"])
    ctx.set_field_grid(0, b["planes0"], nx, float(b["L"]), int(b["ny_period"]))
    ctx.set_field_grid(1, b["planes1"], nx, float(b["L"]), int(b["ny_period"]))
    x, k, _, _ = ctx.leapfrog(b["x0"], b["k0"], float(b["dt"]), int(b["nsteps"]), float(b["f"]),
                              float(b["gH"]), nslots=2, alpha0=float(b["alpha0"]), dalpha=float(b["dalpha"]),
                              bump=float(b["bump"]))
    np.testing.assert_array_equal(x, b["x"])
    np.testing.assert_array_equal(k, b["k"])


def _close_field(a, b, rtol=FIELD_RTOL):
    scale = max(np.abs(b).max(), 1e-300)
    err = np.abs(np.asarray(a) - np.asarray(b)).max() / scale
    assert err <= rtol, f"relative field error {err:.3e} > {rtol:.1e}"


@pytest.mark.parametrize("nx", [8, 16, 32, 64, 256, 512, 1024, 2048, 4096])
def test_g2k_k2g_vs_numpy(ctx, nx):
    """Every FFT shape: one-buffer radix 4 (n <= 1024, odd and even log2 n),
    ping-pong radix 4 (2048, 4096)."""
    X, Y = periodic_grid(nx)
    rng = np.random.default_rng(nx)
    f = np.zeros_like(X)
    for _ in range(20):
        kx, ky = rng.integers(-nx // 2 + 1, nx // 2, 2)
        f += rng.normal() * np.cos(kx * X + ky * Y + rng.uniform(0, 6))
    f += rng.normal(size=f.shape) * 1e-3  # broadband (incl. Nyquist content)
    fk_g = ctx.g2k(f)
    fk_o = orc.g2k(f)
    _close_field(fk_g, fk_o)
    _close_field(ctx.k2g(fk_o), orc.k2g(fk_o))


def test_golden_field_preparation(ctx):
    g = np.load(os.path.join(GOLD, "golden_fields.npz"))
    nx = g["psi_in"].shape[0]
    ctx.set_field_psi(0, g["psi_in"], nx, 2 * np.pi)
    got = ctx.get_field_grid(0, nx)
    for i in range(6):
        _close_field(got[i], g["planes_psi"][i])
    _close_field(ctx.get_psi_grid(0, nx), g["psi"])
    ctx.set_field_qk(0, g["qk"], nx, 2 * np.pi, float(g["K_d2"]))
    got = ctx.get_field_grid(0, nx)
    for i in range(6):
        _close_field(got[i], g["planes_qk"][i])
    ctx.set_field_qk(0, g["qk"], nx, 2 * np.pi, float(g["K_d2"]), shear=0.5)
    got = ctx.get_field_grid(0, nx)
    for i in range(6):
        _close_field(got[i], g["planes_qk_shear"][i])


def test_grid_U_scaled_wavenumbers_two_layer(ctx):
    # qg2layersw_raytrace.m: L = 20, k scaled by 2*pi/L, shear 0.5, 2 layers.
    import swraytracing_amd as sw
    nx, L = 64, 20.0
    kx_, ky_, K2 = orc.wavenumber_grids(nx, L, scale=True)
    rng = np.random.default_rng(5)
    X, Y = periodic_grid(nx, L)
    q1 = np.cos(2 * np.pi * (3 * X + 2 * Y) / L) + 0.3 * np.sin(2 * np.pi * (5 * X - 4 * Y) / L)
    qk = np.stack([orc.g2k(q1), orc.g2k(-q1)], axis=2)
    fo = orc.grid_U(qk, 3.0, K2, kx_, ky_, 0.5)
    fg = sw.grid_U(qk, 3.0, K2, kx_, ky_, 0.5, ctx=ctx)
    for n in orc.FIELD_ORDER:
        assert fg[n].shape == (nx, nx, 2)
        _close_field(fg[n], fo[n])


def test_spectral_scheme_api_matches_oracle(qg_case):
    import swraytracing_amd as sw
    c = qg_case
    psi = orc.k2g(-c["qk"] / (c["K_d2"] + c["K2"]))
    gs = sw.SpectralScheme(c["L"], c["nx"], psi)
    os_ = orc.SpectralSchemeOracle(c["L"], c["nx"], psi)
    P = 33
    x = c["x"][:P].T[None].copy()
    k = c["k"][:P].T[None].copy()
    scaleU = np.abs(os_.fields["u"]).max()
    scaleG = np.abs(os_.fields["ux"]).max()
    np.testing.assert_allclose(gs.U(x), os_.U(x), rtol=0, atol=1e-13 * scaleU)
    gg, go = gs.grad_U(x), os_.grad_U(x)
    for n in ("u_x", "u_y", "v_x", "v_y"):
        np.testing.assert_allclose(gg[n], go[n], rtol=0, atol=1e-13 * scaleG)
    np.testing.assert_allclose(gs.grad_U_times_k(x, k), os_.grad_U_times_k(x, k), rtol=0,
                               atol=1e-12 * scaleG)
    np.testing.assert_allclose(gs.vorticity(x), os_.vorticity(x), rtol=0, atol=1e-12 * scaleG)
    np.testing.assert_allclose(gs.strain(x), os_.strain(x), rtol=0, atol=1e-12 * scaleG)
    sp = gs.streamfunction(x[0, 0], x[0, 1])
    np.testing.assert_allclose(sp, os_.streamfunction(x[0, 0], x[0, 1]), rtol=0,
                               atol=1e-13 * np.abs(psi).max())
    assert gs.U_field["u"].shape == (c["nx"], c["nx"])


def test_ode_symplectic_gpu_vs_oracle(qg_case):
    import swraytracing_amd as sw
    c = qg_case
    psi = orc.k2g(-c["qk"] / (c["K_d2"] + c["K2"]))
    gs = sw.SpectralScheme(c["L"], c["nx"], psi)
    os_ = orc.SpectralSchemeOracle(c["L"], c["nx"], psi)
    P = 40
    x0 = c["x"][:P].T[None].copy()
    k0 = c["k"][:P].T[None].copy()
    T = c["dt"] * 100.5
    xg, kg, tg = sw.ode_symplectic(x0, k0, c["dt"], T, c["f"], 1.0, gs)
    xo, ko, to = orc.ode_symplectic(x0, k0, c["dt"], T, c["f"], 1.0, os_)
    assert xg.shape == xo.shape == (100, 2, P)
    np.testing.assert_array_equal(tg, to)
    np.testing.assert_allclose(xg, xo, rtol=0, atol=TRAJ_ATOL)
    np.testing.assert_allclose(kg, ko, rtol=0, atol=TRAJ_ATOL * 10)
    # same fields -> bit-exact: run the oracle on the GPU's own fields
    snap = orc.GridField({n: v for n, v in gs._fields().items()}, gs.dx)
    xl, kl, hx, hk = orc.leapfrog(x0[0].T, k0[0].T, c["dt"], 99, c["f"], 1.0, snap, bump=orc.BUMP_SW,
                                  save_every=1)
    np.testing.assert_array_equal(xg[1:], np.stack(hx).transpose(0, 2, 1))
    np.testing.assert_array_equal(kg[1:], np.stack(hk).transpose(0, 2, 1))


def test_full_size_subset_parity(ctx, oracle_lib):
    """BASELINE size: 512^2 field, 1e6 packets.  Packets are independent, so
    a random subset run through the oracle must match the GPU bit for bit."""
    nx, L = 512, 2 * np.pi
    rng = np.random.default_rng(146)
    X, Y = periodic_grid(nx, L)
    psi = np.zeros_like(X)
    for _ in range(40):
        kx, ky = rng.integers(-30, 31, 2)
        psi += rng.normal() / (1 + kx * kx + ky * ky) * np.cos(kx * X + ky * Y + rng.uniform(0, 6))
    ctx.set_field_psi(0, psi, nx, L)
    planes = ctx.get_field_grid(0, nx)
    N = 1_000_000
    x, k = orc.initial_packets(N, L, 4.0, 3.0, 1.0, rng)
    ctx.packets_set(x, k)
    dt, steps = 0.004, 12
    ctx.advance(dt, steps, 3.0, 1.0, bump=orc.BUMP_SW)
    xg, kg = ctx.packets_get()
    assert np.isfinite(xg).all() and np.isfinite(kg).all()
    idx = np.sort(rng.choice(N, 3000, replace=False))
    xo, ko, _, _ = oracle_lib.leapfrog(planes, None, 0, 0, nx, nx, L / nx, orc.BUMP_SW, x[idx], k[idx], dt,
                                       steps, 3.0, 1.0)
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)


def test_edge_cases(ctx, qg_case):
    import swraytracing_amd as sw
    c = qg_case
    nx, L = c["nx"], c["L"]
    ctx.set_field_grid(0, _planes(c["flow"]), nx, L)
    # empty ensemble
    x, k, _, _ = ctx.leapfrog(np.zeros((0, 2)), np.zeros((0, 2)), 0.01, 5, 3.0, 1.0)
    assert x.shape == (0, 2)
    # single packet, zero steps
    x1 = np.array([[0.1, 0.2]])
    k1 = np.array([[3.0, -1.0]])
    xs, ks, _, _ = ctx.leapfrog(x1, k1, 0.01, 0, 3.0, 1.0)
    np.testing.assert_array_equal(xs, x1)
    # NaN / Inf packets do not fault and stay non-finite; others unaffected
    xb = np.array([[np.nan, 0.0], [np.inf, 1.0], [0.3, 0.4]])
    kb = np.array([[1.0, 1.0], [1.0, 1.0], [1.0, 2.0]])
    xs, ks, _, _ = ctx.leapfrog(xb, kb, 0.01, 3, 3.0, 1.0)
    assert not np.isfinite(xs[0]).all() and not np.isfinite(xs[1]).all()
    xr, kr, _, _ = ctx.leapfrog(xb[2:], kb[2:], 0.01, 3, 3.0, 1.0)
    np.testing.assert_array_equal(xs[2:], xr)
    # argument errors surface as SwrtError, not crashes
    with pytest.raises(sw.SwrtError):
        ctx.advance(0.01, 1, 3.0, 1.0, nslots=3)
    with pytest.raises(sw.SwrtError):
        ctx.set_field_grid(5, _planes(c["flow"]), nx, L)  # SWRT_MAX_SLOTS = 5
    fresh = sw.Context(0)
    fresh.packets_set(x1, k1)
    with pytest.raises(sw.SwrtError):
        fresh.advance(0.01, 1, 3.0, 1.0)
    fresh.close()


def test_packet_ensemble_driver_frames(tmp_path, qg_case):
    """PacketEnsemble writes packet_x/k/time.bin frames that read_field and
    load_data.m's layout accept (N x 2 column-major per frame, wrapped x)."""
    import swraytracing_amd as sw
    c = qg_case
    nx = c["nx"]
    ens = sw.PacketEnsemble(c["x"], c["k"], c["L"], c["f"], c["Cg"], nx, c["K_d2"])
    qk2 = c["qk"] * 1.01
    ens.set_snapshots(c["qk"], qk2)
    d = str(tmp_path)
    ens.write_frame(0.0, d)
    ens.advance(c["dt"], nsub=4)
    ens.write_frame(c["dt"], d)
    t = sw.read_field(os.path.join(d, "packet_time"))
    assert t.shape == (1, 2)
    xs = sw.read_field(os.path.join(d, "packet_x"), c["x"].shape[0], 2, 1, [1, 2])
    assert xs.shape == (c["x"].shape[0], 2, 2)
    assert np.all(xs >= -c["L"] / 2) and np.all(xs < c["L"] / 2)
    # advance == oracle blend on the GPU-built fields
    fo0 = orc.grid_U(c["qk"], c["K_d2"], c["K2"], c["kx_"], c["ky_"])
    fo1 = orc.grid_U(qk2, c["K_d2"], c["K2"], c["kx_"], c["ky_"])
    xo, ko, _, _ = orc.leapfrog(c["x"], c["k"], c["dt"] / 4, 4, c["f"], 1.0, orc.GridField(fo0, c["L"] / nx),
                                orc.GridField(fo1, c["L"] / nx), 0.125, 0.25, bump=orc.BUMP_QG)
    xg, kg = ens.state()
    np.testing.assert_allclose(xg, xo, rtol=0, atol=TRAJ_ATOL)
    np.testing.assert_allclose(kg, ko, rtol=0, atol=TRAJ_ATOL)


def test_sqrt_div_correctly_rounded_on_device(ctx):
    """Zero-flow drift exercises sqrt and division only: must equal the
    host's IEEE results bit for bit over a wide range of k."""
    nx = 16
    ctx.set_field_grid(0, np.zeros((6, nx * nx)), nx, 2 * np.pi)
    rng = np.random.default_rng(11)
    n = 200000
    k = rng.normal(size=(n, 2)) * np.exp(rng.uniform(-20, 20, (n, 1)))
    x = rng.uniform(-1, 1, (n, 2))
    f, gH, dt = 3.0, 0.7, 0.01
    xg, kg, _, _ = ctx.leapfrog(x, k, dt, 1, f, gH)
    w = np.sqrt(f * f + gH * (k[:, 0] * k[:, 0] + k[:, 1] * k[:, 1]))
    half = dt / 2
    x1 = x + half * (gH * k / w[:, None])
    x2 = x1 + dt * 0.0
    xo = x2 + half * (gH * k / w[:, None])
    np.testing.assert_array_equal(kg, k)
    np.testing.assert_array_equal(xg, xo)


def test_short_ieee_sequences_match_device_ieee(ctx):
    """The hot loop's 10-instruction sqrt, 7-instruction reciprocal and
    one-reciprocal drift (swrt_kernels.hpp sqrt_rn_normal / rcp_rn_normal /
    drift_inc) equal the compiler's IEEE sqrt and division bit for bit over
    6.7e7 random operands per sequence spanning their documented ranges
    (the division quotients' correctness from RN(1/w) is also proven on the
    host: tests/test_divconst.py)."""
    assert ctx.check_arith(1 << 22, seed=7) == (0, 0, 0)


@pytest.mark.parametrize("rebin_every,tile", [(0, 0), (1, 4), (3, 8), (8, 0), (64, 16)])
def test_spatial_binning_is_invisible(ctx, oracle_lib, qg_case, rebin_every, tile):
    """Binning only permutes the device order: final state and history frames
    are bit-identical to the oracle and in the original packet order."""
    c = qg_case
    nx, L = c["nx"], c["L"]
    pl = _planes(c["flow"])
    ctx.set_field_grid(0, pl, nx, L)
    ctx.set_locality(rebin_every, tile)
    try:
        xg, kg, hxg, hkg = ctx.leapfrog(c["x"], c["k"], c["dt"] * 4, 30, c["f"], 1.0, bump=orc.BUMP_SW,
                                        save_every=5)
    finally:
        ctx.set_locality(4, 0)
    xo, ko, hxo, hko = oracle_lib.leapfrog(pl, None, 0, 0, nx, nx, L / nx, orc.BUMP_SW, c["x"], c["k"],
                                           c["dt"] * 4, 30, c["f"], 1.0, save_every=5)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)
    np.testing.assert_array_equal(hxg, hxo)
    np.testing.assert_array_equal(hkg, hko)


@pytest.mark.parametrize("variant", [1, 2])
@pytest.mark.parametrize("nslots", [1, 2])
@pytest.mark.parametrize("dt_scale", [1.0, 40.0])
@pytest.mark.parametrize("div_free", [False, True])
def test_kernel_variants_bitexact(ctx, oracle_lib, qg_case, variant, nslots, dt_scale, div_free):
    """Per-packet (1) and LDS-tiled (2) kernels give
    the oracle's bits; the large-dt case drives packets out of the LDS window
    (global fallback).  div_free: v_y stored as -u_x, so the tile kernel runs
    its five-sum window (swrt_field_div_free); the oracle sums all six."""
    c = qg_case
    nx, L = c["nx"], c["L"]
    p0 = _planes(c["flow"])
    p1 = _planes({n: np.asarray(v) * 0.8 for n, v in c["flow"].items()})
    if div_free:
        p0[5], p1[5] = -p0[2], -p1[2]
    ctx.set_field_grid(0, p0, nx, L, 2 * nx)
    ctx.set_field_grid(1, p1, nx, L, 2 * nx)
    assert ctx.field_div_free(0) is div_free and ctx.field_div_free(1) is div_free
    dt = c["dt"] * dt_scale
    ctx.set_kernel(variant)
    ctx.set_locality(5, 0)
    try:
        xg, kg, hxg, hkg = ctx.leapfrog(c["x"], c["k"], dt, 12, c["f"], 1.0, nslots=nslots, alpha0=0.1,
                                        dalpha=0.07, bump=orc.BUMP_QG, save_every=3)
    finally:
        ctx.set_kernel(0)
        ctx.set_locality(4, 0)
    xo, ko, hxo, hko = oracle_lib.leapfrog(p0, p1 if nslots == 2 else None, 0.1, 0.07, nx, 2 * nx, L / nx,
                                           orc.BUMP_QG, c["x"], c["k"], dt, 12, c["f"], 1.0, save_every=3)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)
    np.testing.assert_array_equal(hxg, hxo)
    np.testing.assert_array_equal(hkg, hko)


@pytest.mark.parametrize("N", [125_000, 20_000])
def test_small_shard_bench_field_bitexact(ctx, oracle_lib, N):
    """A strong-scaling shard of the bench ensemble (1.25e5 = 1e6 / 8 GPUs,
    and a 2e4 tail) on the bench's device-derived 512^2 fields: a random
    subset bit-identical to the C oracle."""
    import argparse
    import bench
    bench._imports()
    args = argparse.Namespace(nx=512, packets=1_000_000, world=8, rank=0, seed=146, mode="blend")
    w = bench.build_workload(ctx, args, 0, N, args.packets)
    ctx.set_locality(20, 0)
    try:
        ctx.packets_set(w["x"], w["k"])
        for _ in range(6):
            bench.step(ctx, w, 5)
        xg, kg = ctx.packets_get()
    finally:
        ctx.set_locality(4, 0)
    p0, p1 = ctx.get_field_grid(0), ctx.get_field_grid(1)
    idx = np.sort(np.random.default_rng(3).choice(N, 2000, replace=False))
    xo, ko = w["x"][idx], w["k"][idx]
    for _ in range(6):
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.1, 0.2, 512, 1024, w["L"] / 512, orc.BUMP_QG, xo, ko,
                                           w["dt"] / 5, 5, w["f"], w["gH"])
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)


def test_broadband_bench_field_bitexact(ctx, oracle_lib):
    """The bench workload on SURVEY §8(d)'s broadband field (bench.py --field
    broadband: |psi| ~ |k|^-3 up to 0.75 kmax, every scale on the 512^2 x 2
    grid): 1e6 packets, 6 calls of 5 steps, a random subset bit-identical to
    the C oracle."""
    import argparse
    import bench
    bench._imports()
    args = argparse.Namespace(nx=512, packets=1_000_000, world=1, rank=0, seed=146, mode="blend",
                              field="broadband")
    w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
    ctx.set_locality(20, 0)
    try:
        ctx.packets_set(w["x"], w["k"])
        for _ in range(6):
            bench.step(ctx, w, 5)
        xg, kg = ctx.packets_get()
    finally:
        ctx.set_locality(4, 0)
    p0, p1 = ctx.get_field_grid(0), ctx.get_field_grid(1)
    idx = np.sort(np.random.default_rng(5).choice(args.packets, 2000, replace=False))
    xo, ko = w["x"][idx], w["k"][idx]
    for _ in range(6):
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.1, 0.2, 512, 1024, w["L"] / 512, orc.BUMP_QG, xo, ko,
                                           w["dt"] / 5, 5, w["f"], w["gH"])
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)


@pytest.mark.parametrize("sparse", [1, 2])
@pytest.mark.parametrize("dt_scale", [1.0, 40.0])
def test_sparse_tiles_bitexact(ctx, oracle_lib, qg_case, sparse, dt_scale):
    """The two-snapshot tile launch in the dense shape (512 threads, reads
    one tap ahead) and the sparse shape (256 threads, 256 VGPRs, reads three
    taps ahead: swrt_set_sparse_tiles 2): the oracle's bits, history frames
    included; dt x 40 drives packets onto the global fallback gather."""
    c = qg_case
    nx, L = c["nx"], c["L"]
    p0 = _planes(c["flow"])
    p1 = _planes({n: np.asarray(v) * 0.8 for n, v in c["flow"].items()})
    p0[5], p1[5] = -p0[2], -p1[2]  # five-sum window
    ctx.set_field_grid(0, p0, nx, L, 2 * nx)
    ctx.set_field_grid(1, p1, nx, L, 2 * nx)
    rng = np.random.default_rng(37)
    N = 3001
    x = (rng.random((N, 2)) - 0.5) * L
    th = rng.random(N) * 2 * np.pi
    k = 3.0 * np.stack([np.cos(th), np.sin(th)], axis=1)
    dt = c["dt"] * dt_scale
    ctx.set_kernel(2)
    ctx.set_locality(5, 0)
    ctx.set_sparse_tiles(sparse)
    try:
        xg, kg, hxg, hkg = ctx.leapfrog(x, k, dt, 12, c["f"], 1.0, nslots=2, alpha0=0.1, dalpha=0.07,
                                        bump=orc.BUMP_QG, save_every=3)
    finally:
        ctx.set_sparse_tiles(0)
        ctx.set_kernel(0)
        ctx.set_locality(4, 0)
    xo, ko, hxo, hko = oracle_lib.leapfrog(p0, p1, 0.1, 0.07, nx, 2 * nx, L / nx, orc.BUMP_QG, x, k, dt, 12,
                                           c["f"], 1.0, save_every=3)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)
    np.testing.assert_array_equal(hxg, hxo)
    np.testing.assert_array_equal(hkg, hko)


@pytest.mark.parametrize("N,sparse", [(125_000, 0), (125_000, 1), (400_000, 2)])
def test_sparse_tiles_bench_field_bitexact(fresh_ctx, oracle_lib, N, sparse):
    """Strong-scaling shards of the bench ensemble on its device-derived 512^2
    fields, 5 substeps per call, re-binning every 20 steps, two packet
    streams: 1.25e5 packets in the automatic (sparse) and the dense shape,
    and 4e5 forced sparse (~390 packets per tile: every lane of a 256-thread
    workgroup takes two packets) — one shape's bits equal the other's, and a
    random subset the C oracle's."""
    import argparse
    import bench
    ctx = fresh_ctx
    bench._imports()
    args = argparse.Namespace(nx=512, packets=1_000_000, world=8, rank=0, seed=146, mode="blend")
    w = bench.build_workload(ctx, args, 0, N, args.packets)
    ctx.set_locality(20, 0)
    ctx.set_sparse_tiles(sparse)
    ctx.packets_set(w["x"], w["k"])
    for _ in range(6):
        bench.step(ctx, w, 5)
    xg, kg = ctx.packets_get()
    p0, p1 = ctx.get_field_grid(0), ctx.get_field_grid(1)
    idx = np.sort(np.random.default_rng(5).choice(N, 2000, replace=False))
    xo, ko = w["x"][idx], w["k"][idx]
    for _ in range(6):
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.1, 0.2, 512, 1024, w["L"] / 512, orc.BUMP_QG, xo, ko,
                                           w["dt"] / 5, 5, w["f"], w["gH"])
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)
    # the other shape, same calls: the same bits for every packet
    ctx.set_sparse_tiles(1 if sparse != 1 else 2)
    ctx.packets_set(w["x"], w["k"])
    for _ in range(6):
        bench.step(ctx, w, 5)
    x2, k2 = ctx.packets_get()
    assert np.array_equal(xg.view(np.uint64), x2.view(np.uint64))
    assert np.array_equal(kg.view(np.uint64), k2.view(np.uint64))


@pytest.mark.parametrize("variant,streams", [(2, 2), (2, 1), (1, 1)])
def test_tile_kernel_large_ensemble_subset(ctx, oracle_lib, variant, streams):
    """512^2 two-snapshot field, 2e5 packets, LDS kernel (one or two packet
    streams) or the per-packet kernel, re-binning every 3 steps over 10 steps:
    random subset bit-identical to the oracle."""
    nx, L = 512, 20.0
    rng = np.random.default_rng(2024)
    kmax = nx // 2 - 1
    qk = np.zeros((2 * kmax + 1, kmax + 1), complex)
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(kmax + 1)[None, :]
    ring = (kx * kx + ky * ky > 100) & (kx * kx + ky * ky <= 900)
    qk[ring] = np.exp(2j * np.pi * rng.random(ring.sum())) * 0.02
    ctx.set_field_qk(0, qk, nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
    ctx.set_field_qk(1, qk * np.exp(0.05j), nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
    p0 = ctx.get_field_grid(0, nx)
    p1 = ctx.get_field_grid(1, nx)
    N = 200_000
    x, k = orc.initial_packets(N, L, 4.0, 3.0, 1.0, rng)
    ctx.set_kernel(variant)
    ctx.set_locality(3, 0)
    ctx.set_packet_streams(streams)
    try:
        ctx.packets_set(x, k)
        ctx.advance(0.01, 10, 3.0, 1.0, nslots=2, alpha0=0.05, dalpha=0.1, bump=orc.BUMP_QG)
        xg, kg = ctx.packets_get()
    finally:
        ctx.set_kernel(0)
        ctx.set_locality(4, 0)
        ctx.set_packet_streams(2)
    idx = np.sort(rng.choice(N, 2000, replace=False))
    xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.05, 0.1, nx, 2 * nx, L / nx, orc.BUMP_QG, x[idx], k[idx], 0.01,
                                       10, 3.0, 1.0)
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)


@pytest.mark.parametrize("variant,sparse", [(1, 0), (2, 1), (2, 2)])
def test_tile_kernel_dense_cluster(ctx, oracle_lib, qg_case, variant, sparse):
    """20000 packets packed into a few cells: tiles far above the
    per-workgroup sort batch (several batches per tile) and
    one-tile-heavy binning; every packet bit-identical to the oracle."""
    c = qg_case
    nx, L = c["nx"], c["L"]
    p0 = _planes(c["flow"])
    p1 = _planes({n: np.asarray(v) * 0.9 for n, v in c["flow"].items()})
    ctx.set_field_grid(0, p0, nx, L, 2 * nx)
    ctx.set_field_grid(1, p1, nx, L, 2 * nx)
    rng = np.random.default_rng(77)
    N = 20_000
    dxg = L / nx
    x = np.stack([rng.random(N) * 3 * dxg + 5.2 * dxg, rng.random(N) * 3 * dxg - 9.7 * dxg], axis=1)
    th = rng.random(N) * 2 * np.pi
    k = 3.0 * np.stack([np.cos(th), np.sin(th)], axis=1)
    ctx.set_kernel(variant)
    ctx.set_locality(2, 0)
    ctx.set_sparse_tiles(sparse)
    try:
        xg, kg, _, _ = ctx.leapfrog(x, k, c["dt"], 9, c["f"], 1.0, nslots=2, alpha0=0.2, dalpha=0.05,
                                    bump=orc.BUMP_QG)
    finally:
        ctx.set_sparse_tiles(0)
        ctx.set_kernel(0)
        ctx.set_locality(4, 0)
    xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.2, 0.05, nx, 2 * nx, L / nx, orc.BUMP_QG, x, k, c["dt"], 9,
                                       c["f"], 1.0)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)


@pytest.mark.parametrize("variant", [2, 1])
def test_tile_kernel_single_step_calls(ctx, oracle_lib, qg_case, variant):
    """One advance call per step (the bench's pattern): with re-binning every
    4 steps, 3 of 4 launches read packets in the cell order the previous
    launch wrote (no in-tile sort); every packet stays bit-identical."""
    c = qg_case
    nx, L = c["nx"], c["L"]
    p0 = _planes(c["flow"])
    p1 = _planes({n: np.asarray(v) * 1.1 for n, v in c["flow"].items()})
    ctx.set_field_grid(0, p0, nx, L, 2 * nx)
    ctx.set_field_grid(1, p1, nx, L, 2 * nx)
    rng = np.random.default_rng(5)
    N = 6000
    x = (rng.random((N, 2)) - 0.5) * L
    th = rng.random(N) * 2 * np.pi
    k = 3.0 * np.stack([np.cos(th), np.sin(th)], axis=1)
    a0, da, nst = 0.05, 0.09, 11
    ctx.set_kernel(variant)
    ctx.set_locality(4, 0)
    try:
        ctx.packets_set(x, k)
        for s in range(nst):
            ctx.advance(c["dt"] * 3, 1, c["f"], 1.0, nslots=2, alpha0=a0 + s * da, dalpha=da, bump=orc.BUMP_QG)
        xg, kg = ctx.packets_get()
    finally:
        ctx.set_kernel(0)
    xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, a0, da, nx, 2 * nx, L / nx, orc.BUMP_QG, x, k, c["dt"] * 3, nst,
                                       c["f"], 1.0)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)


def _rsw_background(nx, seed=3):
    """Childress-Soward flow (ray_trace_sw/raytrace.m:30-37) + a smooth H."""
    U, G = orc.childress_soward(nx, U0=0.1, km=4.0, a=0.25)
    X, Y = periodic_grid(nx)
    H = 1.0 + 0.1 * np.cos(2 * X + Y) + 0.05 * np.sin(3 * Y)
    return U, G, H


@pytest.mark.parametrize("nx", [32, 64])
def test_step_packet_xka_bitexact(ctx, nx):
    """GPU step_packet_xka (cg_sw per tap) == the literal full-field oracle."""
    import swraytracing_amd as sw
    U, G, H = _rsw_background(nx)
    dx = 2 * np.pi / nx
    rng = np.random.default_rng(nx)
    npk, steps, dt, C0, f = 24, 6, 0.3 * dx, 1.0, 4.0
    P0 = {"x": rng.uniform(0, 2 * np.pi, npk), "y": rng.uniform(-7, 7, npk),
          "k": 40 * np.cos(np.arange(npk)), "l": 40 * np.sin(np.arange(npk)), "a": np.ones(npk)}
    hist = sw.raytrace_xka(P0, U, G, H, C0, f, dx, dx, dt, steps, ctx=ctx)
    for i in range(npk):
        P = {n: float(P0[n][i]) for n in "xykla"}
        for j in range(1, steps):
            P = orc.step_packet_xka(P, U, G, H, C0, f, dx, dx, dt)
            for n in "xykla":
                assert hist[n][i, j] == P[n], (i, j, n, hist[n][i, j], P[n])


@pytest.mark.parametrize("nx,steps", [(64, 6), (1024, 9)])
def test_step_packet_xka_binned_order_is_invisible(ctx, nx, steps):
    """Ensembles >= 4096 packets are stepped in spatially binned order by the
    LDS-tiled kernel (swrt_xka_step; 8x8-cell tiles at 64^2, 16x16 at 1024^2),
    re-binned every 4 steps: final states and every history frame are
    bit-identical to the unbinned lane order of the per-packet kernel (itself
    pinned to the literal oracle above), and the first packets match the
    oracle directly."""
    import swraytracing_amd as sw
    U, G, H = _rsw_background(nx)
    dx = 2 * np.pi / nx
    rng = np.random.default_rng(11)
    npk, dt, C0, f = 6000, 0.3 * dx, 1.0, 4.0
    P0 = {"x": rng.uniform(0, 2 * np.pi, npk), "y": rng.uniform(-7, 7, npk),
          "k": 40 * np.cos(np.arange(npk)), "l": 40 * np.sin(np.arange(npk)), "a": np.ones(npk)}
    ctx.set_locality(4, 0)
    binned = sw.raytrace_xka(P0, U, G, H, C0, f, dx, dx, dt, steps, ctx=ctx)
    ctx.set_locality(0, 0)
    try:
        plain = sw.raytrace_xka(P0, U, G, H, C0, f, dx, dx, dt, steps, ctx=ctx)
    finally:
        ctx.set_locality(4, 0)
    for n in "xykla":
        np.testing.assert_array_equal(binned[n], plain[n])
    for i in range(3):
        P = {n: float(P0[n][i]) for n in "xykla"}
        for j in range(1, steps):
            P = orc.step_packet_xka(P, U, G, H, C0, f, dx, dx, dt)
            for n in "xykla":
                assert binned[n][i, j] == P[n]


@pytest.mark.parametrize("save_every", [3, 8])
def test_xka_binned_history_frames_any_save_every(ctx, save_every):
    """Binned xka launches are cut every rebin_every (4) steps; frames are
    picked by the global step, so save_every need not divide the launch
    length: every frame equals the unbinned single-launch path's."""
    nx = 64
    U, G, H = _rsw_background(nx)
    dx = 2 * np.pi / nx
    rng = np.random.default_rng(12)
    n, dt, nsteps = 6000, 0.3 * dx, 24
    st = np.stack([rng.uniform(0, 2 * np.pi, n), rng.uniform(-7, 7, n), 40 * np.cos(np.arange(n)),
                   40 * np.sin(np.arange(n)), np.ones(n)], axis=1)
    ctx.xka_set_fields(U, G, H, dx, dx)
    ctx.set_locality(4, 0)
    sb, hb = ctx.xka_step(st, 1.0, 4.0, dt, nsteps, save_every)
    ctx.set_locality(0, 0)
    try:
        sp, hp = ctx.xka_step(st, 1.0, 4.0, dt, nsteps, save_every)
    finally:
        ctx.set_locality(4, 0)
    assert hb.shape == (nsteps // save_every, n, 5)
    np.testing.assert_array_equal(sb, sp)
    np.testing.assert_array_equal(hb, hp)
    np.testing.assert_array_equal(hb[-1], sb)


def test_xka_zero_steps_leaves_state(ctx):
    """nsteps == 0 on a binned-size ensemble: no launch, state unchanged."""
    nx = 64
    U, G, H = _rsw_background(nx)
    dx = 2 * np.pi / nx
    rng = np.random.default_rng(13)
    n = 6000
    st = np.stack([rng.uniform(0, 2 * np.pi, n), rng.uniform(0, 2 * np.pi, n), rng.normal(size=n),
                   rng.normal(size=n), np.ones(n)], axis=1)
    ctx.xka_set_fields(U, G, H, dx, dx)
    ctx.set_locality(4, 0)
    s0, h0 = ctx.xka_step(st, 1.0, 4.0, 0.1 * dx, 0, 0)
    assert h0 is None
    np.testing.assert_array_equal(s0, st)


def test_step_packet_xka_scalar_api(ctx):
    import swraytracing_amd as sw
    nx = 32
    U, G, H = _rsw_background(nx)
    dx = 2 * np.pi / nx
    P = {"x": 0.3, "y": 1.7, "k": 12.0, "l": -5.0, "a": 2.0}
    g = sw.step_packet_xka(P, U, G, H, 1.0, 4.0, dx, dx, 0.02, ctx=ctx)
    o = orc.step_packet_xka(P, U, G, H, 1.0, 4.0, dx, dx, 0.02)
    assert g == o


def test_omega_histogram_matches_load_data(ctx):
    """analysis/load_data.m:33-52,63: omega, histcounts (last bin closed), mean."""
    rng = np.random.default_rng(31)
    n = 300_000
    k = rng.normal(size=(n, 2)) * 5
    x = rng.uniform(-3, 3, (n, 2))
    ctx.packets_set(x, k)
    f, Cg = 3.0, 1.0
    w = np.sqrt(f ** 2 + Cg ** 2 * (k * k).sum(1))
    edges = np.linspace(0, w.max(), 300)  # load_data.m:38-39 (bins = 300 edges)
    counts, mean = ctx.omega_histogram(f, Cg, edges)
    ref, _ = np.histogram(w, edges)
    np.testing.assert_array_equal(counts, ref)
    assert counts.sum() == n  # max sits on the closed last edge
    assert abs(mean - w.mean()) < 1e-12 * w.mean()
    # accumulation over frames (load_data.m windows)
    counts2, _ = ctx.omega_histogram(f, Cg, edges, counts.copy())
    np.testing.assert_array_equal(counts2, 2 * ref)


@pytest.mark.parametrize("n_cells", [1, 3])
def test_fma_gather_mode_tolerance(ctx, oracle_lib, n_cells):
    """swrt_set_gather_mode(1): the stencil sums and the snapshot blend by
    fused multiply-add (one rounding per tap instead of two).  Tolerance
    parity against the bit-exact oracle on the bench's device-derived 512^2
    fields (five-sum window): <= 1e-13 relative per step over 20 steps
    (k, |x|); the default mode stays bit-identical (same launch, mode 0)."""
    import argparse
    import bench
    bench._imports()
    args = argparse.Namespace(nx=512, packets=200_000, world=1, rank=0, seed=146, mode="blend")
    w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
    assert ctx.field_div_free(0) and ctx.field_div_free(1)
    nsteps, sub = 20, 5
    # n_cells = 3: a 3x longer step, so some packets leave the LDS window (global FMA fallback)
    h = w["dt"] / sub * n_cells
    ctx.set_locality(20, 0)
    out = {}
    try:
        for mode in (1, 0):
            ctx.set_gather_mode(mode)
            ctx.packets_set(w["x"], w["k"])
            for _ in range(nsteps // sub):
                ctx.advance(h, sub, w["f"], w["gH"], nslots=2, alpha0=0.5 / sub, dalpha=1.0 / sub, bump=orc.BUMP_QG)
            out[mode] = ctx.packets_get()
    finally:
        ctx.set_gather_mode(0)
        ctx.set_locality(4, 0)
    p0, p1 = ctx.get_field_grid(0), ctx.get_field_grid(1)
    idx = np.sort(np.random.default_rng(9).choice(args.packets, 2000, replace=False))
    xo, ko = w["x"][idx], w["k"][idx]
    for _ in range(nsteps // sub):
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.5 / sub, 1.0 / sub, 512, 1024, w["L"] / 512, orc.BUMP_QG,
                                           xo, ko, h, sub, w["f"], w["gH"])
    np.testing.assert_array_equal(out[0][0][idx], xo)   # mode 0: bit-exact
    np.testing.assert_array_equal(out[0][1][idx], ko)
    xf, kf = out[1][0][idx], out[1][1][idx]
    tol = nsteps * 1e-13
    assert np.abs(xf - xo).max() <= tol * np.abs(xo).max()
    assert np.abs(kf - ko).max() <= tol * np.abs(ko).max()
    assert not np.array_equal(xf, xo)  # the FMA path really ran


def test_packet_streams_bit_identical(fresh_ctx, oracle_lib):
    """swrt_set_packet_streams(2 / 4): tile launches as two half (four
    quarter) launches on two (four) streams, joined only when something reads
    the packets.  A call sequence that mixes history frames, re-binnings
    inside and between calls, a field rewrite, multi-interval launches, reads
    and ode23 gives the bits of one stream — and the oracle's on a subset."""
    ctx = fresh_ctx
    import argparse
    import bench
    import swraytracing_amd as sw
    bench._imports()
    args = argparse.Namespace(nx=512, packets=300_000, world=1, rank=0, seed=146, mode="blend")
    w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
    p0, p1 = ctx.get_field_grid(0).copy(), ctx.get_field_grid(1).copy()
    h = w["dt"] / 5
    out = {}
    for streams in (2, 1):
        ctx.set_packet_streams(streams)
        ctx.set_locality(20, 0)
        try:
            ctx.set_field_grid(0, p0, 512, w["L"], 1024)
            ctx.set_field_grid(1, p1, 512, w["L"], 1024)
            ctx.packets_set(w["x"], w["k"])
            ctx.history_reset()
            for _ in range(7):  # 35 steps: re-binnings at 20 and inside a call at 40 > 35
                ctx.advance(h, 5, w["f"], w["gH"], nslots=2, alpha0=0.1, dalpha=0.2, bump=orc.BUMP_QG, save_every=5)
            x1, k1 = ctx.packets_get()
            hx, hk = ctx.history()
            ctx.set_field_grid(1, p0, 512, w["L"], 1024)  # rewrite a slot the second stream read
            ctx.set_field_grid(2, p1, 512, w["L"], 1024)
            ctx.advance_intervals([h, 1.1 * h], 5, w["f"], w["gH"], alpha0=0.1, dalpha=0.2, bump=orc.BUMP_QG)
            ctx.advance(h, 3, w["f"], w["gH"], nslots=2, alpha0=0.1, dalpha=0.2, bump=orc.BUMP_QG)
            x2, k2 = ctx.packets_get()
            ctx.set_field_grid(1, p1, 512, w["L"], 1024)
            st = {}
            sw.ode23_packets(ctx, (0.0, 5 * h), 5 * h, w["f"], 1.0, stats=st)
            x3, k3 = ctx.packets_get()
            out[streams] = (x1, k1, hx, hk, x2, k2, x3, k3)
        finally:
            ctx.set_packet_streams(2)  # the library default
            ctx.set_locality(4, 0)
    for streams in (2,):
        for a, b in zip(out[1], out[streams]):
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), streams
    idx = np.sort(np.random.default_rng(4).choice(args.packets, 1500, replace=False))
    xo, ko = w["x"][idx], w["k"][idx]
    for _ in range(7):
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.1, 0.2, 512, 1024, w["L"] / 512, orc.BUMP_QG, xo, ko, h, 5,
                                           w["f"], w["gH"])
    np.testing.assert_array_equal(out[2][0][idx], xo)
    np.testing.assert_array_equal(out[2][1][idx], ko)


def test_packet_streams_long_run_bit_identical(fresh_ctx):
    """The bench workload (1e6 packets, 5 substeps per call, re-binning every
    20 steps) over 100 calls — 25 re-binnings, each followed by a sort launch
    that gathers its input from any slot while the parts of the split launch
    run on 2 streams — gives every packet's bits of one stream."""
    ctx = fresh_ctx
    import argparse
    import bench
    bench._imports()
    args = argparse.Namespace(nx=512, packets=1_000_000, world=1, rank=0, seed=146, mode="blend")
    w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
    out = {}
    try:
        ctx.set_locality(20, 0)
        for streams in (1, 2):
            ctx.set_packet_streams(streams)
            ctx.packets_set(w["x"], w["k"])
            for _ in range(100):
                bench.step(ctx, w, 5)
            out[streams] = ctx.packets_get()
    finally:
        ctx.set_packet_streams(2)
        ctx.set_locality(4, 0)
    for streams in (2,):
        for a, b in zip(out[1], out[streams]):
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), streams


@pytest.mark.parametrize("substeps,rebin_every,calls", [(5, 20, 10), (1, 4, 12)])
def test_bench_configuration_subset_bitexact(fresh_ctx, oracle_lib, substeps, rebin_every, calls):
    """The headline bench configuration itself (bench.py: 2-layer 512^2 field,
    L = 20, shear 0.5, two snapshots, 1e6 packets, one advance call per PDE
    interval of `substeps` leapfrog steps — the default 5 steps of
    0.05*dx/U0 with re-binning every 20, and the single-step 0.25*dx/U0 form
    with re-binning every 4 — the default kernel): a random subset of 3000
    packets bit-identical to the C oracle on the same device-prepared fields."""
    ctx = fresh_ctx
    import argparse
    import bench
    bench._imports()
    args = argparse.Namespace(nx=512, packets=1_000_000, world=1, rank=0, seed=146, mode="blend")
    ctx.set_locality(rebin_every, 0)
    ctx.set_kernel(0)
    try:
        w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
        ctx.packets_set(w["x"], w["k"])
        for _ in range(calls):
            bench.step(ctx, w, substeps)
        xg, kg = ctx.packets_get()
        p0 = ctx.get_field_grid(0, 512)
        p1 = ctx.get_field_grid(1, 512)
    finally:
        ctx.set_locality(4, 0)
    idx = np.sort(np.random.default_rng(7).choice(args.packets, 3000, replace=False))
    xo, ko = w["x"][idx], w["k"][idx]
    for _ in range(calls):  # bench.step: substeps leapfrog steps of dt/substeps, alpha = (s + 1/2)/substeps
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.5 / substeps, 1.0 / substeps, 512, 1024, w["L"] / 512,
                                           orc.BUMP_QG, xo, ko, w["dt"] / substeps, substeps, w["f"], w["gH"])
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)


def test_div_free_detection_and_derived_fields(ctx, qg_case):
    """Host fields are divergence-free only if v_y == -u_x bit for bit (a
    one-ulp change at one node turns it off); fields derived on the device
    from psi / qk store v_y = -u_x, and that v_y agrees with the oracle's
    separately transformed one within FIELD_RTOL (grid_U.m:9,17)."""
    c = qg_case
    nx, L = c["nx"], c["L"]
    p = _planes(c["flow"])
    p[5] = -p[2]
    ctx.set_field_grid(0, p, nx, L)
    assert ctx.field_div_free(0)
    p[5, 17] = np.nextafter(p[5, 17], np.inf)
    ctx.set_field_grid(0, p, nx, L)
    assert not ctx.field_div_free(0)
    X, Y = periodic_grid(nx)
    psi = np.sin(3 * X + Y) + 0.3 * np.cos(X - 5 * Y) + 0.1 * np.sin(7 * Y)
    ctx.set_field_psi(0, psi, nx, 2 * np.pi)
    assert ctx.field_div_free(0)
    g = ctx.get_field_grid(0, nx)
    np.testing.assert_array_equal(g[5], -g[2])
    want = orc.spectral_scheme_fields(2 * np.pi, nx, psi)
    _close_field(g[5], np.asarray(want["vy"]).ravel(order="F"))


@pytest.mark.timeout(120)
def test_cli_driver_runs_the_bench_workload():
    """The C-ABI command-line driver (no Python in the loop) runs the bench
    workload at reduced size and reports finite packets and a throughput."""
    import json
    import subprocess
    cli = os.path.join(ROOT, "build", "bin", "swrt_cli")
    assert os.path.exists(cli), "swrt_cli not built"
    r = subprocess.run([cli, "--nx", "256", "--packets", "100000", "--steps", "8", "--warmup", "2"],
                       capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["finite"] is True and d["value"] > 0 and d["steps"] == 8


@pytest.mark.timeout(120)
def test_maximum_size_ensemble_subset():
    """Largest configuration of BASELINE.json (configs[4]'s sizes): a 1024^2
    two-snapshot field and 1e7 packets through the default LDS tile kernel
    (4096 tiles, half-tile tail, bench-style calls of 5 substeps, re-binning
    every 20 over a 40-step run): every packet finite, a random subset of
    2000 bit-identical to the C oracle on the device-prepared fields."""
    import swraytracing_amd as sw
    from oracle import cbind
    nx, L, N = 1024, 20.0, 10_000_000
    rng = np.random.default_rng(99)
    kmax = nx // 2 - 1
    qk = np.zeros((2 * kmax + 1, kmax + 1), complex)
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(kmax + 1)[None, :]
    ring = (kx * kx + ky * ky > 100) & (kx * kx + ky * ky <= 900)
    qk[ring] = np.exp(2j * np.pi * rng.random(ring.sum())) * 0.01
    ctx = sw.Context(0)
    try:
        ctx.set_field_qk(0, qk, nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
        ctx.set_field_qk(1, qk * np.exp(0.03j), nx, L, 3.0, 0.5, 2 * np.pi / L, 2 * nx)
        p0 = ctx.get_field_grid(0, nx)
        p1 = ctx.get_field_grid(1, nx)
        U0 = float(np.sqrt((p0[0] ** 2 + p0[1] ** 2).max()))
        dt = 0.25 * (L / nx) / U0
        x = (rng.random((N, 2)) - 0.5) * L
        th = rng.random(N) * 2 * np.pi
        k = np.sqrt(15.0) * 3.0 * np.stack([np.cos(th), np.sin(th)], axis=1)
        ctx.set_locality(20, 0)
        ctx.packets_set(x, k)
        sub, calls = 5, 8
        for _ in range(calls):
            ctx.advance(dt / sub, sub, 3.0, 1.0, nslots=2, alpha0=0.5 / sub, dalpha=1.0 / sub, bump=orc.BUMP_QG)
        xg, kg = ctx.packets_get()
    finally:
        ctx.close()
    assert np.isfinite(xg).all() and np.isfinite(kg).all()
    idx = np.sort(rng.choice(N, 2000, replace=False))
    xo, ko = x[idx], k[idx]
    for _ in range(calls):
        xo, ko, _, _ = cbind.leapfrog(p0, p1, 0.5 / sub, 1.0 / sub, nx, 2 * nx, L / nx, orc.BUMP_QG, xo, ko,
                                      dt / sub, sub, 3.0, 1.0)
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)


@pytest.mark.parametrize("sparse", [0, 1])
def test_tile_path_non_finite_and_far_packets(fresh_ctx, oracle_lib, sparse):
    """Bad inputs on the LDS-tiled hot path (the bench field, 70,000 packets,
    two packet streams, 8 calls of 5 steps with re-binning every 20; the
    automatic launch shape at ~68 packets per tile is the sparse one, 1 forces
    the dense one): packets
    at NaN / +-Inf positions or with a NaN wavevector are binned, sorted and
    advanced without a fault and stay non-finite; packets far outside the
    periodic domain (|x| ~ 1e6 L, interpolate.m's mod wraps them) and exactly
    on its edges match the C oracle bit for bit; every other packet is
    bit-identical to the run without the bad ones (packets never interact,
    ode_symplectic.m:18-21)."""
    import argparse
    import bench
    ctx = fresh_ctx
    bench._imports()
    args = argparse.Namespace(nx=512, packets=70_000, world=1, rank=0, seed=146, mode="blend")
    w = bench.build_workload(ctx, args, 0, args.packets, args.packets)
    x, k = w["x"].copy(), w["k"].copy()
    L = w["L"]
    bad = {10: (np.nan, 0.0), 20: (np.inf, 1.0), 30: (0.0, -np.inf)}
    far = {40: (1e6 * L + 0.3, -2.5e6 * L), 50: (-L / 2, -L / 2), 60: (L / 2, L / 2 - 1e-13)}
    for i, v in {**bad, **far}.items():
        x[i] = v
    k[70] = (np.nan, 1.0)
    ctx.set_locality(20, 0)
    ctx.set_sparse_tiles(sparse)
    out = {}
    try:
        for name, xs in (("mixed", x), ("clean", w["x"])):
            ks = k if name == "mixed" else w["k"]
            ctx.packets_set(xs, ks)
            for _ in range(8):
                bench.step(ctx, w, 5)
            out[name] = ctx.packets_get()
        p0, p1 = ctx.get_field_grid(0, 512), ctx.get_field_grid(1, 512)
    finally:
        ctx.set_locality(4, 0)
    xg, kg = out["mixed"]
    for i in (10, 20, 30, 70):
        assert not (np.isfinite(xg[i]).all() and np.isfinite(kg[i]).all()), i
    special = [10, 20, 30, 40, 50, 60, 70]
    keep = np.setdiff1d(np.arange(args.packets), special)
    assert xg[keep].tobytes() == out["clean"][0][keep].tobytes()
    assert kg[keep].tobytes() == out["clean"][1][keep].tobytes()
    idx = np.array(sorted(far))
    xo, ko = x[idx], k[idx]
    for _ in range(8):
        xo, ko, _, _ = oracle_lib.leapfrog(p0, p1, 0.1, 0.2, 512, 1024, L / 512, orc.BUMP_QG, xo, ko,
                                           w["dt"] / 5, 5, w["f"], w["gH"])
    np.testing.assert_array_equal(xg[idx], xo)
    np.testing.assert_array_equal(kg[idx], ko)
