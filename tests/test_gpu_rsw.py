"""GPU field preparation against MATLAB's own arrays, and the RSW background
of step_packet_xka (ray_trace_sw/raytrace_sw.m:16-52) on the device.

* swrt_g2k / swrt_k2g against `rsw/matlab.mat`'s Sk, Sout and u/v/h/zeta
  (tests/golden/gen_rsw_mat.py), at FIELD_RTOL — the same arrays pin the CPU
  oracle in tests/test_matlab_pins.py.
* swrt_xka_set_rsw against the oracle's rsw_background at FIELD_RTOL, on a
  balanced 2-D state plus MATLAB's wave (whose geostrophic part vanishes).
* step_packet_xka trajectories over the device-built background, bit-exact
  against the literal full-field oracle run on the same (downloaded) fields.
"""
import os

import numpy as np
import pytest

from oracle import swrt_oracle as orc
from tests.test_matlab_pins import balanced_state

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIELD_RTOL = 1e-13  # FFT round-off relative to the field's max (as test_gpu_parity)


@pytest.fixture(scope="module")
def mat():
    return dict(np.load(os.path.join(GOLDEN, "rsw_matlab.npz")))


def _rel(a, b):
    return np.abs(np.asarray(a) - np.asarray(b)).max() / np.abs(b).max()


@pytest.mark.parametrize("i,name", [(0, "u"), (1, "v"), (2, "h")])
def test_device_g2k_k2g_match_matlab(ctx, mat, i, name):
    Sk = mat["Sk"][:, :, i]
    assert _rel(ctx.g2k(mat[name]), Sk) <= FIELD_RTOL          # g2k.m vs swk.m:113
    assert _rel(ctx.k2g(Sk), mat["Sout"][:, :, i, 3]) <= FIELD_RTOL  # k2g.m vs swk.m:146
    assert _rel(ctx.k2g(ctx.g2k(mat["Sin"][:, :, i])), mat["Sout"][:, :, i, 0]) <= FIELD_RTOL


def test_device_derivative_convention_matches_matlab(ctx, mat):
    kx_, ky_, _ = orc.wavenumber_grids(256)
    Sk = mat["Sk"]
    assert _rel(ctx.k2g(1j * kx_ * Sk[:, :, 1] - 1j * ky_ * Sk[:, :, 0]), mat["zeta"]) <= FIELD_RTOL


def _fields_close(ctx, bg):
    U, G, H = ctx.xka_get_fields()
    for name in "uv":
        assert _rel(U[name], bg["U"][name]) <= FIELD_RTOL, name
    for name in ("u_x", "u_y", "v_x", "v_y"):
        assert _rel(G[name], bg["GradU"][name]) <= FIELD_RTOL, name
    # H = 1 + etag: compare etag against its own scale
    assert np.abs((H - 1.0) - bg["etag"]).max() <= FIELD_RTOL * np.abs(bg["etag"]).max()
    return U, G, H


@pytest.mark.parametrize("nx", [64, 256])
def test_xka_set_rsw_matches_oracle(ctx, mat, nx):
    f, Cg = 1.0, 1.0
    S = balanced_state(nx, f, Cg, seed=nx)
    if nx == 256:
        S = S + np.stack([mat["u"], mat["v"], mat["h"]], axis=2)
    ctx.xka_set_rsw(S, f, Cg)
    _fields_close(ctx, orc.rsw_background(S, f, Cg))


def test_xka_set_rsw_other_parameters(ctx):
    # f = 3, Cg = 0.5 (gH0 = Cg^2 != Cg): the projection's f and gH0 enter separately
    f, Cg, nx = 3.0, 0.5, 128
    rng = np.random.default_rng(5)
    S = balanced_state(nx, f, Cg, seed=3) + 0.01 * rng.normal(size=(nx, nx, 3))
    ctx.xka_set_rsw(S, f, Cg)
    _fields_close(ctx, orc.rsw_background(S, f, Cg))


def test_xka_set_rsw_non_2pi_period(ctx):
    """L = 20: wavenumbers scaled by 2*pi/L on the device as in the oracle
    (raytrace_sw.m itself uses L = 2*pi); dx = L/nx for the packet steps."""
    f, Cg, nx, L = 2.0, 1.0, 64, 20.0
    S = balanced_state(nx, f, Cg, seed=9)
    ctx.xka_set_rsw(S, f, Cg, L)
    bg = orc.rsw_background(S, f, Cg, L)
    _fields_close(ctx, bg)
    # the 2*pi fields differ: the scaling is real
    assert _rel(orc.rsw_background(S, f, Cg)["GradU"]["u_x"], bg["GradU"]["u_x"]) > 1e-3


def test_matlab_wave_has_no_geostrophic_background_on_device(ctx, mat):
    S = np.stack([mat["u"], mat["v"], mat["h"]], axis=2)
    ctx.xka_set_rsw(S, 1.0, 1.0)
    U, G, H = ctx.xka_get_fields()
    assert max(np.abs(U["u"]).max(), np.abs(U["v"]).max()) <= 1e-9 * np.abs(S[:, :, :2]).max()
    np.testing.assert_allclose(H, 1.0, atol=1e-10)


def test_raytrace_sw_trajectories_bitexact_on_device_background(ctx, mat):
    """raytrace_sw.m's packet loop over the device-built background: each
    packet's trajectory equals the literal step_packet_xka oracle on the same
    field bits (downloaded), step for step."""
    import swraytracing_amd as sw
    f, Cg, nx = 1.0, 1.0, 256
    S = balanced_state(nx, f, Cg, amp=0.1, seed=7) + np.stack([mat["u"], mat["v"], mat["h"]], axis=2)
    dx = 2 * np.pi / nx
    kd = f / Cg
    ki = 10 * kd  # raytrace_sw.m:85-86
    npk, steps = 10, 8  # np = 10 (raytrace_sw.m:97)
    rng = np.random.default_rng(123)
    i = np.arange(1, npk + 1)
    P0 = {"x": rng.uniform(0, 2 * np.pi, npk), "y": rng.uniform(0, 2 * np.pi, npk),
          "k": ki * np.cos(2 * np.pi * i / npk), "l": ki * np.sin(2 * np.pi * i / npk), "a": np.ones(npk)}
    U0 = np.sqrt(S[:, :, 0] ** 2 + S[:, :, 1] ** 2).max()
    dt = 0.3 * dx / max(Cg, U0)  # raytrace_sw.m:100
    hist = sw.raytrace_sw(S, f, Cg, P0, dt, steps, ctx=ctx)
    U, G, H = ctx.xka_get_fields()
    for p in range(npk):
        P = {n: float(P0[n][p]) for n in "xykla"}
        for j in range(1, steps):
            P = orc.step_packet_xka(P, U, G, H, Cg, f, dx, dx, dt)
            for n in "xykla":
                assert hist[n][p, j] == P[n], (p, j, n)
    # the action changes (div C != 0 over a non-uniform H) and stays positive
    assert np.all(hist["a"][:, -1] > 0) and np.any(hist["a"][:, -1] != 1.0)
