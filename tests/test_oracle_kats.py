"""Pin the CPU oracle against analytic known answers (CPU only).

The reference ships no numeric vectors, so these KATs are what
pins the restatement: each asserts a property the reference algorithm must
have, derived from the cited .m files."""
import math

import numpy as np
import pytest

from oracle import swrt_oracle as orc
from tests.conftest import periodic_grid


def test_lagrange_weights_sum_and_partition():
    # interpolate.m:33-41 — the (j - i) denominator makes each 1-D set sum to
    # -1 (odd number of sign flips), while the 2-D product sums to +1.
    a = np.linspace(0.0, 0.999, 37)
    w = orc.lagrange_weights(a, 0.0)
    s = sum(w)
    np.testing.assert_allclose(s, -1.0, rtol=0, atol=1e-13)
    np.testing.assert_allclose(sum(wi * wj for wi in w for wj in w), 1.0, atol=1e-13)
    # at a = 0 (bump 0) the stencil is exact at node i = 0 (with sign -1)
    w0 = orc.lagrange_weights(np.array([0.0]), 0.0)
    assert w0[2][0] == -1.0 and all(w0[i][0] == 0.0 for i in (0, 1, 3, 4, 5))


def test_matlab_mod_semantics():
    m = 64.0
    a = np.array([-1e-17, -64.0, -0.5, 0.0, 63.999999, 64.0, 130.25, -200.75])
    r = orc.matlab_mod(a, m)
    assert np.all(r >= 0) and np.all(r <= m)
    np.testing.assert_array_equal(r[[1, 3, 5]], [0.0, 0.0, 0.0])
    assert r[0] == 64.0  # round-up case: a - floor(a/m)*m rounds to m
    np.testing.assert_allclose(r[[2, 6, 7]], [63.5, 2.25, 55.25])


def test_interpolate_reproduces_degree5_polynomial_periodic_shift():
    # 6-point Lagrange interpolation is exact for trigonometric-free data that
    # is locally polynomial of degree <= 5; use a smooth periodic field and
    # check the 6th-order convergence and shift invariance by nx*dx.
    for nx in (32, 64):
        L = 2 * np.pi
        X, Y = periodic_grid(nx, L)
        F = np.sin(X) * np.cos(2 * Y)
        rng = np.random.default_rng(0)
        x = rng.uniform(-10, 10, 200)
        y = rng.uniform(-10, 10, 200)
        FI = orc.interpolate(x, y, F, L / nx, L / nx, bump=0.0)
        err = np.abs(FI - np.sin(x) * np.cos(2 * y)).max()
        assert err < (6e-5 if nx == 32 else 2e-6), err
        FI2 = orc.interpolate(x + L, y - 2 * L, F, L / nx, L / nx, bump=0.0)
        np.testing.assert_allclose(FI2, FI, atol=1e-12)


def test_k2g_g2k_roundtrip_and_point_formula():
    nx = 32
    X, Y = periodic_grid(nx)
    f = np.cos(3 * X + 2 * Y + 0.3) + 0.5 * np.sin(-5 * X + 7 * Y) + 0.25
    fk = orc.g2k(f)
    assert fk.shape == (nx - 1, nx // 2)
    np.testing.assert_allclose(orc.k2g(fk), f, atol=1e-14)
    # f(x,y) = Re fk(0,0) + sum 2 Re(fk e^{i(kx x + ky y)})
    kmax = nx // 2 - 1
    x0, y0 = 0.7, -1.3
    val = fk[kmax, 0].real
    for r in range(2 * kmax + 1):
        for c in range(kmax + 1):
            kx, ky = r - kmax, c
            if (ky == 0 and kx > 0) or ky > 0:
                val += 2 * (fk[r, c] * np.exp(1j * (kx * x0 + ky * y0))).real
    exact = math.cos(3 * x0 + 2 * y0 + 0.3) + 0.5 * math.sin(-5 * x0 + 7 * y0) + 0.25
    assert abs(val - exact) < 1e-13


def test_grid_U_single_mode_is_exact():
    # psi = A cos(Kx + Ly + ph): grid_U's derivative spectra give the exact
    # u = -psi_y, v = psi_x and gradients at the nodes.
    nx, K, Lw, A, ph = 32, 3, 2, 0.7, 0.4
    X, Y = periodic_grid(nx)
    psi = A * np.cos(K * X + Lw * Y + ph)
    sch = orc.spectral_scheme_fields(2 * np.pi, nx, psi)
    s = np.sin(K * X + Lw * Y + ph)
    c = np.cos(K * X + Lw * Y + ph)
    np.testing.assert_allclose(sch["u"], A * Lw * s, atol=1e-13)
    np.testing.assert_allclose(sch["v"], -A * K * s, atol=1e-13)
    np.testing.assert_allclose(sch["ux"], A * Lw * K * c, atol=1e-12)
    np.testing.assert_allclose(sch["uy"], A * Lw * Lw * c, atol=1e-12)
    np.testing.assert_allclose(sch["vx"], -A * K * K * c, atol=1e-12)
    np.testing.assert_allclose(sch["vy"], -A * K * Lw * c, atol=1e-12)
    # grid_U with qk of the same psi (q = -(K_d2 + K^2) psi)
    kx_, ky_, K2 = orc.wavenumber_grids(nx)
    K_d2 = 3.0
    qk = -orc.g2k(psi) * (K_d2 + K2)
    fl = orc.grid_U(qk, K_d2, K2, kx_, ky_, 0.5)
    np.testing.assert_allclose(fl["u"], A * Lw * s + 0.5, atol=1e-13)
    np.testing.assert_allclose(fl["vx"], -A * K * K * c, atol=1e-12)


def test_zero_flow_drift_is_exact():
    # Config 1 (SW_zero_background_raytracing): U = 0 -> phi2 is the identity,
    # x(t) advances by the group velocity each half step, k constant.
    nx = 32
    z = {n: np.zeros((nx, nx)) for n in orc.FIELD_ORDER}
    rng = np.random.default_rng(5)
    x, k = orc.initial_packets(256, 2 * np.pi, 4.0, 3.0, 1.0, rng)
    dt, f, gH = 0.01, 3.0, 1.0
    xs, ks, _, _ = orc.leapfrog(x, k, dt, 50, f, gH, orc.GridField(z, 2 * np.pi / nx))
    np.testing.assert_array_equal(ks, k)
    w = np.sqrt(f * f + gH * (k[:, 0] ** 2 + k[:, 1] ** 2))
    cg = gH * k / w[:, None]
    np.testing.assert_allclose(xs, x + 50 * dt * cg, rtol=0, atol=1e-12)


def test_fourier_exact_kick_matches_grid_kick():
    # scratch/fourier_interpolate_test.m:92-114 (exact kick of a random n=5
    # Fourier field) vs the gridded SpectralScheme kick: same to 6th-order
    # interpolation error (SURVEY §8c KAT iv).
    n = 5
    rng = np.random.default_rng(44)
    N = 2 * n + 1
    amp = 0.5 * rng.random((N, N)) / N**2
    phase = 2 * np.pi * rng.random((N, N))
    nx = 128  # fourier_interpolate_test.m:4
    X, Y = periodic_grid(nx)
    psi = orc.fourier_streamfunction(X, Y, amp, phase, n)
    sch = orc.SpectralSchemeOracle(2 * np.pi, nx, psi, bump=0.0)
    x0 = rng.uniform(-np.pi, np.pi, (300, 2))
    k0 = rng.normal(size=(300, 2)) * 3
    dt = 0.01
    xe, ke = orc.fourier_phi2(x0, k0, dt, amp, phase, n)
    X3 = x0.T[None]
    K3 = k0.T[None]
    xg = X3 + dt * sch.U(X3)
    kg = K3 - dt * sch.grad_U_times_k(X3, K3)
    np.testing.assert_allclose(xg[0].T, xe, atol=3e-9)
    np.testing.assert_allclose(kg[0].T, ke, atol=3e-8)
    # and the closed-form gradient helper agrees with the exact kick
    ux, uy, vx, vy = orc.fourier_grad(x0[:, 0], x0[:, 1], amp, phase, n)
    kk = k0 - dt * np.stack([ux * k0[:, 0] + vx * k0[:, 1], uy * k0[:, 0] + vy * k0[:, 1]], axis=1)
    np.testing.assert_allclose(kk, ke, atol=1e-14)


def test_single_mode_absolute_frequency_conservation():
    # images/Symplectic_error/single_fourier_mode.png: |d omega_a / omega_0|
    # stays ~1e-5 for a single Fourier mode with the leapfrog integrator.
    nx, A, K, Lw = 64, 0.05, 1, 1
    X, Y = periodic_grid(nx)
    psi = A * np.cos(K * X + Lw * Y)
    sch = orc.SpectralSchemeOracle(2 * np.pi, nx, psi)
    f, gH = 3.0, 1.0
    rng = np.random.default_rng(123)
    P = 8
    x0 = np.zeros((1, 2, P)); k0 = np.zeros((1, 2, P))
    for i in range(P):
        k0[0, :, i] = 3 * np.array([math.cos(2 * math.pi * (i + 1) / P), math.sin(2 * math.pi * (i + 1) / P)])
        x0[0, :, i] = 2 * np.pi * rng.random(2) - np.pi
    xs, ks, t = orc.ode_symplectic(x0, k0, 0.05, 20.0, f, gH, sch)
    Om = np.sqrt(f * f + gH * np.sum(ks * ks, axis=1)) + np.sum(sch.U(xs) * ks, axis=1)
    rel = np.abs(Om - Om[0:1]) / Om[0:1]
    assert rel.max() < 5e-5, rel.max()


def test_numpy_and_c_oracles_bit_identical(oracle_lib, qg_case):
    c = qg_case
    pl = oracle_lib.planes_of(c["flow"])
    snap = orc.GridField(c["flow"], c["L"] / c["nx"])
    xn, kn, hx, hk = orc.leapfrog(c["x"], c["k"], c["dt"], 12, c["f"], 1.0, snap, bump=1e-13, save_every=4)
    xc, kc, hxc, hkc = oracle_lib.leapfrog(pl, None, 0, 0, c["nx"], c["nx"], c["L"] / c["nx"], 1e-13,
                                          c["x"], c["k"], c["dt"], 12, c["f"], 1.0, save_every=4)
    np.testing.assert_array_equal(xn, xc)
    np.testing.assert_array_equal(kn, kc)
    np.testing.assert_array_equal(np.stack(hx).transpose(0, 2, 1), hxc)
    # two-snapshot blend + 2-layer y-period
    fl2 = {n: v * 1.05 for n, v in c["flow"].items()}
    s2 = orc.GridField(fl2, c["L"] / c["nx"], 2 * c["nx"])
    s1 = orc.GridField(c["flow"], c["L"] / c["nx"], 2 * c["nx"])
    xn, kn, _, _ = orc.leapfrog(c["x"], c["k"], c["dt"], 6, c["f"], 1.0, s1, s2, 0.1, 0.2, bump=1e-10)
    xc, kc, _, _ = oracle_lib.leapfrog(pl, oracle_lib.planes_of(fl2), 0.1, 0.2, c["nx"], 2 * c["nx"],
                                       c["L"] / c["nx"], 1e-10, c["x"], c["k"], c["dt"], 6, c["f"], 1.0)
    np.testing.assert_array_equal(xn, xc)
    np.testing.assert_array_equal(kn, kc)


def test_cpu_arranged_leapfrog_bit_identical(oracle_lib, qg_case, tmp_path):
    """oracle_leapfrog_fast (bench.py's cpu_baseline: interleaved padded nodes,
    weights shared by both snapshots, drift increment once per step) gives
    the restatement's bits, also as the -O3 -march=native build that bench.py
    compiles on the host it times."""
    c = qg_case
    pl = oracle_lib.planes_of(c["flow"])
    pl2 = oracle_lib.planes_of({n: v * 0.93 for n, v in c["flow"].items()})
    L = c["L"]
    rng = np.random.default_rng(9)
    x = np.concatenate([c["x"], (rng.random((64, 2)) - 0.5) * 3 * L])  # far outside the period too
    k = np.concatenate([c["k"], c["k"][:64]])
    cpu, _flags = oracle_lib.cpu_lib(str(tmp_path))
    for p1, nyF, a0, da in [(None, c["nx"], 0.0, 0.0), (pl2, 2 * c["nx"], 0.1, 0.07)]:
        xr, kr, _, _ = oracle_lib.leapfrog(pl, p1, a0, da, c["nx"], nyF, L / c["nx"], 1e-10, x, k, c["dt"] * 7,
                                           9, c["f"], 1.0)
        for lib in (None, cpu):
            xf, kf = oracle_lib.leapfrog_fast(pl, p1, a0, da, c["nx"], nyF, L / c["nx"], 1e-10, x, k,
                                              c["dt"] * 7, 9, c["f"], 1.0, L=lib)
            np.testing.assert_array_equal(xf, xr)
            np.testing.assert_array_equal(kf, kr)


def test_ode_symplectic_layout_and_leapfrog_equivalence(qg_case):
    c = qg_case
    sch = orc.SpectralSchemeOracle(c["L"], c["nx"], orc.k2g(-c["qk"] / (c["K_d2"] + c["K2"])))
    P = 7
    x0 = c["x"][:P].T[None].copy()
    k0 = c["k"][:P].T[None].copy()
    X, K, t = orc.ode_symplectic(x0, k0, c["dt"], c["dt"] * 9.5, c["f"], 1.0, sch)
    assert X.shape == (9, 2, P) and t.shape == (9,)
    np.testing.assert_array_equal(X[0], x0[0])
    np.testing.assert_allclose(t, np.arange(9) * c["dt"])
    xl, kl, hx, hk = orc.leapfrog(c["x"][:P], c["k"][:P], c["dt"], 8, c["f"], 1.0,
                                  orc.GridField(sch.fields, sch.dx), bump=1e-13, save_every=1)
    np.testing.assert_array_equal(X[1:], np.stack(hx).transpose(0, 2, 1))
    np.testing.assert_array_equal(K[1:], np.stack(hk).transpose(0, 2, 1))


def test_two_layer_interpolate_reads_layer1_with_2nx_period():
    # CS3: interpolate on an nx x nx x 2 F: ny = 2*nx in the y-mod, layer 1 read.
    nx = 32
    X, Y = periodic_grid(nx)
    F = np.zeros((nx, nx, 2))
    F[:, :, 0] = np.sin(X + 2 * Y)
    F[:, :, 1] = 99.0
    rng = np.random.default_rng(3)
    x = rng.uniform(-20, 20, 100)
    y = rng.uniform(-20, 20, 100)
    a = orc.interpolate(x, y, F, 2 * np.pi / nx, 2 * np.pi / nx, bump=1e-10)
    b = orc.interpolate(x, y, F[:, :, 0], 2 * np.pi / nx, 2 * np.pi / nx, bump=1e-10)
    np.testing.assert_allclose(a, b, atol=1e-12)
    assert np.abs(a).max() < 1.5
