"""GPU exact spectral evaluator (SURVEY K3 / scratch/fourier_interpolate_test.m)
vs the oracle's direct sincos sum.  Not a rounding-order restatement (the
reference has no production code for it), so compared within tolerance:
  fp64: <= 1e-12 of the field's max magnitude (phase recurrence over <= 511
        modes per row, re-seeded every row);
  fp32: the config-5 envelope at 1024^2 (test_config5_fp32_envelope_1024):
        positions within steps*dt*e_U, wavevectors within steps*dt*e_gradU
        (e_* = the fp32 evaluation error of U / grad U at the start points),
        at most linear growth, and the same absolute-frequency drift as fp64;
        full table in profiles/r02_config5_fp32_study.json (tools/fp32_study.py)."""
import numpy as np
import pytest

from oracle import swrt_oracle as orc
from tests.conftest import periodic_grid

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return np.abs(a - b).max() / np.abs(b).max()


def test_amp_phase_field_matches_exact_kick(ctx):
    n = 5
    rng = np.random.default_rng(44)
    N = 2 * n + 1
    amp = 0.5 * rng.random((N, N)) / N**2
    phase = 2 * np.pi * rng.random((N, N))
    C, kx0, ky0, s = orc.modes_from_amp_phase(amp, phase, n)
    ctx.spectral_set_modes(C, kx0, ky0, s)
    x0 = rng.uniform(-np.pi, np.pi, (500, 2))
    k0 = rng.normal(size=(500, 2)) * 3
    I = ctx.spectral_eval(x0[:, 0], x0[:, 1], 64)
    O = orc.spectral_direct(C, kx0, ky0, s, x0[:, 0], x0[:, 1])
    for q in range(6):
        assert _rel(I[q], O[q]) < 1e-12
    # exact kick of fourier_interpolate_test.m:92-114
    dt = 0.01
    xe, ke = orc.fourier_phi2(x0, k0, dt, amp, phase, n)
    xg = x0 + dt * I[0:2].T
    kg = k0 - dt * np.stack([I[2] * k0[:, 0] + I[4] * k0[:, 1], I[3] * k0[:, 0] + I[5] * k0[:, 1]], axis=1)
    np.testing.assert_allclose(xg, xe, rtol=0, atol=1e-15)
    np.testing.assert_allclose(kg, ke, rtol=0, atol=1e-14)


@pytest.mark.parametrize("nx", [64, 256])
def test_halfplane_spectrum_vs_direct_sum_and_grid(ctx, nx):
    X, Y = periodic_grid(nx)
    rng = np.random.default_rng(nx)
    psi = np.zeros_like(X)
    for _ in range(30):
        kx, ky = rng.integers(-nx // 8, nx // 8, 2)  # <= 0.8 rad/cell: 6-point Lagrange accurate to ~1e-4
        psi += rng.normal() / (1 + kx * kx + ky * ky) * np.cos(kx * X + ky * Y + rng.uniform(0, 6))
    fk = orc.g2k(psi)
    C, kx0, ky0, s = orc.modes_from_halfplane(fk)
    ctx.spectral_set_modes(C, kx0, ky0, s)
    x = rng.uniform(-10, 10, 300)
    y = rng.uniform(-10, 10, 300)
    I64 = ctx.spectral_eval(x, y, 64)
    O = orc.spectral_direct(C, kx0, ky0, s, x, y)
    for q in range(6):
        assert _rel(I64[q], O[q]) < 1e-12, q
    I32 = ctx.spectral_eval(x, y, 32)
    err32 = max(_rel(I32[q], O[q]) for q in range(6))
    assert err32 < 1e-3, err32
    # exact evaluation agrees with the gridded SpectralScheme to interpolation error
    sch = orc.SpectralSchemeOracle(2 * np.pi, nx, psi)
    G = orc.interpolate_fields(x, y, sch.fields, sch.dx, 1e-13)
    for q in range(6):
        assert _rel(I64[q], G[q]) < 1e-3


def test_spectral_leapfrog_matches_oracle(ctx):
    import swraytracing_amd as sw
    nx = 64
    X, Y = periodic_grid(nx)
    psi = 0.05 * np.cos(2 * X + Y + 0.3) + 0.02 * np.sin(-3 * X + 4 * Y)
    sch = sw.FourierScheme.from_halfplane(orc.g2k(psi), ctx=ctx)
    C, kx0, ky0, s = orc.modes_from_halfplane(orc.g2k(psi))
    rng = np.random.default_rng(7)
    x = rng.uniform(-3, 3, (128, 2))
    k = rng.normal(size=(128, 2)) * 4
    f, gH, dt, steps = 3.0, 1.0, 0.01, 50
    xg, kg = sch.leapfrog(x, k, dt, steps, f, gH)
    xo, ko = x.copy(), k.copy()
    for _ in range(steps):
        w = np.sqrt(f * f + gH * (ko[:, 0] ** 2 + ko[:, 1] ** 2))
        x1 = xo + dt / 2 * (gH * ko / w[:, None])
        I = orc.spectral_direct(C, kx0, ky0, s, x1[:, 0], x1[:, 1])
        x2 = x1 + dt * I[0:2].T
        k2 = ko - dt * np.stack([I[2] * ko[:, 0] + I[4] * ko[:, 1], I[3] * ko[:, 0] + I[5] * ko[:, 1]], axis=1)
        w = np.sqrt(f * f + gH * (k2[:, 0] ** 2 + k2[:, 1] ** 2))
        xo = x2 + dt / 2 * (gH * k2 / w[:, None])
        ko = k2
    np.testing.assert_allclose(xg, xo, rtol=0, atol=1e-12)
    np.testing.assert_allclose(kg, ko, rtol=0, atol=1e-11)
    # Omega_abs conservation in the steady exact field (symplectic_full_fourier.m:41,54-57)
    def Om(xx, kk):
        I = orc.spectral_direct(C, kx0, ky0, s, xx[:, 0], xx[:, 1])
        return np.sqrt(f * f + gH * (kk ** 2).sum(1)) + I[0] * kk[:, 0] + I[1] * kk[:, 1]
    # leapfrog keeps a shadow Hamiltonian: O(dt^2) oscillation, no drift (cf. the
    # ~2.5e-3 level of images/Symplectic_error/second_order_symplectic_error_dt=0.05.png)
    assert (np.abs(Om(xg, kg) - Om(x, k)) / Om(x, k)).max() < 2e-3


def test_config5_fp32_envelope_1024(ctx):
    """BASELINE configs[4] (symplectic_full_fourier.m:20,37,44 at 1024^2, a
    65k subset of the 1e7-packet ensemble): fp32 and fp64 exact-kick leapfrog
    side by side over 64 steps of dt = 0.1*dx/max(Cg, U0).  Envelope:
      per-step bound  max|x32 - x64|(s) <= 2 * s * dt * e_U
                      max|k32 - k64|(s) / max|k| <= 2 * s * dt * e_gradU
      growth          error(64) / error(8) <= 8  (no faster than linear)
      science         |drift32 - drift64| <= 1e-8 of the relative Omega_abs
                      drift (symplectic_full_fourier.m:54-57)."""
    from tools.fp32_study import study
    r = study(ctx, nx=1024, stride=153, chunks=8, per_chunk=8)
    dt, eU, eG = r["dt"], r["fp32_eval_err_U"], r["fp32_eval_err_gradU"]
    assert 0 < eU < 1e-5 and 0 < eG < 1e-4, (eU, eG)
    tab = r["table"]
    for row in tab:
        s = row["steps"]
        assert row["max_abs_x_err"] <= 2 * s * dt * eU, row
        assert row["max_rel_k_err"] <= 2 * s * dt * eG, row
        assert abs(row["omega_abs_drift_fp32"] - row["omega_abs_drift_fp64"]) <= 1e-8, row
        assert row["omega_abs_drift_fp64"] < 1e-3  # leapfrog shadow-Hamiltonian level
    assert tab[-1]["max_abs_x_err"] <= 8 * tab[0]["max_abs_x_err"]
    assert tab[-1]["max_rel_k_err"] <= 8 * tab[0]["max_rel_k_err"]
