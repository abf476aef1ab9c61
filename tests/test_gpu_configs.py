"""BASELINE.json's configurations, each at its stated size, on the GPU path.

  configs[0] SW_zero_background_raytracing.m: 256 packets, U = 0 .... here
  configs[1] steady single-layer QG, 256^2 field, 1e4 packets ........ here
  configs[2] stored PV snapshots, 512^2, 1e5 packets ...... tests/test_gpu_stored.py
  configs[3] two-layer QG, 512^2 x 2, 1e6 packets ......... tests/test_gpu_parity.py
             (test_bench_configuration_subset_bitexact), tests/test_gpu_qg.py
             (test_qg2_driver_loop_512_matches_oracle_pipeline), the bench
  configs[4] 1024^2, 1e7 packets, fp32 study .............. tests/test_gpu_spectral.py,
             tests/test_gpu_parity.py::test_maximum_size_ensemble_subset

Parity: bit-exact against the C oracle (oracle/swrt_oracle.c, the restatement
of interpolate.m:18-49, interpolate_U.m:19-23 and ode_symplectic.m:10-28), and
for U = 0 against the closed form of the drift.
"""
import numpy as np
import pytest

from oracle import swrt_oracle as orc

pytestmark = pytest.mark.gpu


def test_config0_zero_background_256_packets(fresh_ctx, oracle_lib):
    """configs[0] (SW_zero_background_raytracing.m, parameters of
    qgsw_raytrace.m:13-60: f = 3, Cg = 1, omega0 = 4f, L = 2 pi): 256 packets
    through a zero flow.  The kick is the identity, so each leapfrog step is
    two half drifts at the packet's fixed group velocity gH k/omega(k):
    k unchanged bit for bit, x equal to the C oracle bit for bit and to
    x0 + t gH k/omega to round-off of the step count."""
    import swraytracing_amd as sw
    ctx = fresh_ctx
    nx, L, f, Cg, N, nsteps = 64, 2 * np.pi, 3.0, 1.0, 256, 400
    zero = np.zeros((6, nx * nx))
    ctx.set_field_grid(0, zero, nx, L)
    rng = np.random.default_rng(146)
    x, k = orc.initial_packets(N, L, 4.0, f, Cg, rng)
    dt = 0.05 * (L / nx) / 0.2
    xg, kg, _, _ = ctx.leapfrog(x, k, dt, nsteps, f, Cg * Cg, nslots=1, bump=sw.BUMP_QG)
    xo, ko, _, _ = oracle_lib.leapfrog(zero, None, 0.0, 0.0, nx, nx, L / nx, orc.BUMP_QG, x, k, dt, nsteps, f,
                                       Cg * Cg)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)
    assert np.array_equal(kg, k)
    om = np.sqrt(f * f + Cg * Cg * (k ** 2).sum(axis=1))
    exact = x + (nsteps * dt) * (Cg * Cg) * k / om[:, None]
    assert np.abs(xg - exact).max() <= 4 * nsteps * np.finfo(float).eps * np.abs(exact).max()


def test_config1_steady_qg_256_1e4_packets(fresh_ctx, oracle_lib):
    """configs[1]: a steady single-layer QG background on a 256^2 grid
    (qgsw_raytrace.m:13-70: initial_q's 5 < |k| <= 8 ring normalised to
    max|U| = 0.2, grid_U on the device from the spectrum), 1e4 packets on
    the omega0 = 4f ring, 100 leapfrog steps of 0.05 dx/U0 in calls of 5
    (re-binning every 20): every packet bit-identical to the C oracle on the
    device-prepared field."""
    import swraytracing_amd as sw
    ctx = fresh_ctx
    nx, L, f, Cg, N = 256, 2 * np.pi, 3.0, 1.0, 10_000
    rng = np.random.default_rng(146)
    q = orc.initial_q(nx, L, 0.2, f / Cg, 5, 8, rng)
    ctx.set_field_qk(0, orc.g2k(q), nx, L, f / Cg, 0.0)
    p0 = ctx.get_field_grid(0, nx)
    U0 = float(np.sqrt((p0[0] ** 2 + p0[1] ** 2).max()))
    x, k = orc.initial_packets(N, L, 4.0, f, Cg, rng)
    dt = 0.05 * (L / nx) / U0
    ctx.set_locality(20, 0)
    try:
        ctx.packets_set(x, k)
        for _ in range(20):
            ctx.advance(dt, 5, f, Cg * Cg, nslots=1, bump=sw.BUMP_QG)
        xg, kg = ctx.packets_get()
    finally:
        ctx.set_locality(4, 0)
    xo, ko, _, _ = oracle_lib.leapfrog(p0, None, 0.0, 0.0, nx, nx, L / nx, orc.BUMP_QG, x, k, dt, 100, f, Cg * Cg)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)
    assert np.isfinite(xg).all()
