"""Known-answer tests of the QG PDE oracle (oracle/swrt_oracle.py QG1Oracle /
QG2Oracle; qgsw_raytrace.m:111-137,270-286, qg2layersw_raytrace.m:129-181).

The reference ships no PDE fixtures, so the oracle is pinned analytically:
* a single Fourier mode has J(psi, q) = 0 (all gradients are parallel), so
  1 layer: qk is unchanged without forcing / filter, and scaled by Ef^n with
  the filter; 2 layers: qk(n dt) = expm(n dt factor_L) qk(0) (scipy expm, an
  independent route from the oracle's pageeig LV diag(exp) LV^-1);
* the spectral Jacobian of two modes equals the analytic product;
* AB3 with a constant tendency integrates it exactly.
"""
import math

import numpy as np
import pytest
import scipy.linalg

from oracle import swrt_oracle as orc


def _single_mode(nx, kx, ky, amp, layers=1):
    kmax = nx // 2 - 1
    qk = np.zeros((2 * kmax + 1, kmax + 1) + ((layers,) if layers > 1 else ()), dtype=complex)
    if layers == 1:
        qk[kx + kmax, ky] = amp
    else:
        for l in range(layers):
            qk[kx + kmax, ky, l] = amp[l]
    return qk


def test_qg1_single_mode_is_steady_without_forcing():
    nx = 32
    qk0 = _single_mode(nx, 3, 2, 0.7 - 0.2j)
    m = orc.QG1Oracle(qk0, nx, K_d2=3.0, r_drag=0.0, force_strength=0.0, use_filter=False)
    for _ in range(5):
        m.step(0.02)
    np.testing.assert_allclose(m.qk, qk0, atol=1e-14)


def test_qg1_filter_scales_each_step():
    nx = 32
    kx, ky = 11, 9  # kstar = sqrt(11^2+9^2)*dx > 0.75*pi: inside the filtered band
    qk0 = _single_mode(nx, kx, ky, 0.5 + 0.1j)
    m = orc.QG1Oracle(qk0, nx, K_d2=3.0, r_drag=0.0, force_strength=0.0, use_filter=True)
    Ef = orc.qg_filter(*orc.wavenumber_grids(nx)[:2], 2 * math.pi / nx)
    kmax = nx // 2 - 1
    e = Ef[kx + kmax, ky]
    assert e < 1.0
    for _ in range(4):
        m.step(0.02)
    np.testing.assert_allclose(m.qk[kx + kmax, ky], qk0[kx + kmax, ky] * e ** 4, rtol=1e-13)


def test_qg1_constant_tendency_integrates_exactly():
    """With qk = 0 and no J, Qn = r_drag*K2 + forces every step, and the AB
    start-up (Euler, AB2, AB3) integrates a constant exactly: qk = n*dt*Qn."""
    nx = 16
    kmax = nx // 2 - 1
    qk0 = np.zeros((2 * kmax + 1, kmax + 1), complex)
    m = orc.QG1Oracle(qk0, nx, K_d2=3.0, r_drag=0.1, force_strength=0.0, use_filter=False)
    dt = 0.01
    m.step(dt)
    _, _, K2 = orc.wavenumber_grids(nx)
    np.testing.assert_allclose(m.qk.real, dt * 0.1 * K2, rtol=1e-12, atol=1e-15)


def test_qg2_single_mode_matches_expm():
    nx, L = 32, 20.0
    kx, ky = 4, 3
    qk0 = _single_mode(nx, kx, ky, [0.4 + 0.3j, -0.2 + 0.5j], layers=2)
    m = orc.QG2Oracle(qk0, nx, L, K_d2=3.0, shear_strength=0.5)
    dt = 0.05
    n = 6
    for _ in range(n):
        m.step(dt)
    kmax = nx // 2 - 1
    Lmat = m.ops["factor_L"][:, :, kx + kmax, ky]
    want = scipy.linalg.expm(n * dt * Lmat) @ qk0[kx + kmax, ky, :]
    np.testing.assert_allclose(m.qk[kx + kmax, ky, :], want, rtol=1e-11)
    others = m.qk.copy()
    others[kx + kmax, ky, :] = 0
    assert np.abs(others).max() < 1e-14


def test_qg2_expL_matches_expm_everywhere():
    nx, L = 16, 20.0
    ops = orc.qg2_operators(nx, L, 3.0, 0.0, 0.5, 0.1 * (L / nx) ** 8, 4, 0.4)
    E = orc.qg2_expL(ops, 0.03)
    for i in range(ops["K2"].shape[0]):
        for j in range(ops["K2"].shape[1]):
            want = scipy.linalg.expm(0.03 * ops["factor_L"][:, :, i, j])
            np.testing.assert_allclose(E[:, :, i, j], want, rtol=1e-10, atol=1e-14)


def test_spectral_jacobian_of_two_modes():
    """J = psi_x q_y - psi_y q_x for psi = cos(a.x), q = cos(b.x): compare the
    k2g-of-ik products used by update with the analytic grid product."""
    nx = 32
    kmax = nx // 2 - 1
    a, b = (2, 1), (1, 3)
    psik = np.zeros((2 * kmax + 1, kmax + 1), complex)
    qk = np.zeros_like(psik)
    psik[a[0] + kmax, a[1]] = 0.5  # cos = (e^{i} + e^{-i})/2, half plane holds the +k half
    qk[b[0] + kmax, b[1]] = 0.5
    kx_, ky_, _ = orc.wavenumber_grids(nx)
    J = orc._jacobian_term(psik, qk, kx_, ky_)
    xs = np.arange(nx) * 2 * np.pi / nx
    X, Y = np.meshgrid(xs, xs, indexing="ij")
    pa = a[0] * X + a[1] * Y
    pb = b[0] * X + b[1] * Y
    psix, psiy = -a[0] * np.sin(pa), -a[1] * np.sin(pa)
    qx, qy = -b[0] * np.sin(pb), -b[1] * np.sin(pb)
    np.testing.assert_allclose(J, psix * qy - psiy * qx, atol=1e-12)


@pytest.mark.parametrize("layers", [1, 2])
def test_qg_oracle_random_field_stays_finite(layers):
    nx = 32
    rng = np.random.default_rng(3)
    if layers == 1:
        q = orc.initial_q(nx, 2 * np.pi, 0.2, 3.0, 5, 8, rng)
        m = orc.QG1Oracle(orc.g2k(q), nx, 3.0)
        for _ in range(10):
            m.step(0.05 * (2 * np.pi / nx) / 0.2)
    else:
        q = orc.initial_q(nx, 20.0, 0.2, 3.0, 3, 6, rng)
        m = orc.QG2Oracle(np.stack([orc.g2k(q), orc.g2k(-q)], axis=2), nx, 20.0, 3.0)
        for _ in range(10):
            m.step()
    assert np.isfinite(m.qk).all()


# ---------------------------------------------------------------------------
# ode23 restatement (oracle.ode23; MATLAB's own ode23 is unpinned)
# ---------------------------------------------------------------------------
def test_ode23_exponential_decay_within_tolerance():
    st = {}
    ts, y = orc.ode23(lambda t, y: -y, [0.0, 1.0], np.array([1.0, 2.0]), stats=st)
    np.testing.assert_allclose(y, np.exp(-1.0) * np.array([1.0, 2.0]), rtol=1e-4)
    assert ts[0] == 0.0 and ts[-1] == 1.0
    assert st["steps"] >= 10  # MaxStep = 0.1*|tspan| bounds every step


def test_ode23_constant_rhs_is_exact():
    """y' = c: every stage combination reproduces c, the error estimate is 0
    (sum E = 0) and the solution is y0 + t*c up to the additions' round-off."""
    c = np.array([0.3, -1.2, 2.0])
    ts, y = orc.ode23(lambda t, y: c.copy(), [0.0, 2.0], np.zeros(3))
    np.testing.assert_allclose(y, 2.0 * c, rtol=1e-13)


def test_ode23_raytracing_rhs_zero_flow_is_linear_drift():
    """SW_zero_background_raytracing config (U = 0): x(t) = x0 + t*Cg*k/omega(k), k fixed."""
    nx = 16
    zero = {n: np.zeros((nx, nx)) for n in orc.FIELD_ORDER}
    f, Cg = 3.0, 1.0
    rhs = orc.raytracing_rhs(zero, zero, f, Cg, 1.0, 2 * np.pi / nx)
    rng = np.random.default_rng(0)
    x0 = rng.random((20, 2))
    k0 = rng.normal(size=(20, 2)) * 3
    y0 = np.concatenate([x0[:, 0], x0[:, 1], k0[:, 0], k0[:, 1]])
    ts, y = orc.ode23(rhs, [0.0, 0.7], y0)
    om = np.sqrt(f ** 2 + Cg ** 2 * (k0 ** 2).sum(1))
    want = x0 + 0.7 * Cg * k0 / om[:, None]
    np.testing.assert_allclose(y[:20], want[:, 0], rtol=1e-13)
    np.testing.assert_allclose(y[20:40], want[:, 1], rtol=1e-13)
    np.testing.assert_array_equal(y[40:], y0[40:])


# ---------------------------------------------------------------------------
# committed fixtures (tests/golden/gen_golden.py) reproduce exactly
# ---------------------------------------------------------------------------
def _gold(name):
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", name))


def test_golden_qg_fixture_reproduces():
    import importlib.util
    import os
    spec = importlib.util.spec_from_file_location(
        "gen_golden", os.path.join(os.path.dirname(__file__), "golden", "gen_golden.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    fresh = gen.qg_fixture()
    g = _gold("golden_qg.npz")
    for key in ("qk1_0", "qk1_8", "qk2_0", "qk2_8", "dts2"):
        np.testing.assert_array_equal(fresh[key], g[key])


def test_golden_ode23_fixture_reproduces():
    g = _gold("golden_ode23.npz")
    nx = int(g["nx"])
    fl = lambda p: {n: p[i].reshape((nx, nx), order="F") for i, n in enumerate(orc.FIELD_ORDER)}
    rhs = orc.raytracing_rhs(fl(g["planes0"]), fl(g["planes1"]), float(g["f"]), float(g["Cg"]),
                             float(g["tmax"]), float(g["L"]) / nx, nyF=int(g["ny_period"]))
    x0, k0 = g["x0"], g["k0"]
    ts, y = orc.ode23(rhs, [0.0, float(g["tmax"])], np.concatenate([x0[:, 0], x0[:, 1], k0[:, 0], k0[:, 1]]))
    np.testing.assert_array_equal(ts, g["ts"])
    np.testing.assert_array_equal(y, g["y"])
