"""Tracing through stored PV snapshots (BASELINE configs[2]) on the GPU.

A pv.bin / pv_time.bin series written by the product's qgsw_raytrace driver
at 512^2 (write_field.m layout) is traced by trace_stored with 1e5 packets:
* swrt_set_field_q (device g2k + grid_U) equals swrt_g2k + swrt_set_field_qk
  bit for bit, and the oracle's grid_U(g2k(q)) at the FFT tolerance;
* the packets equal the C oracle's leapfrog with interpolate_U's blend run
  over the same field bits (downloaded per frame), interval by interval —
  bit-exact;
* 1 and 4 intervals per call give the same bits.
Reference: read_field.m:37-98, symplectic_full_fourier.m:18-20,
interpolate_U.m:19-23, grid_U.m:1-18."""
import math

import numpy as np
import pytest

import swraytracing_amd as sw
from oracle import swrt_oracle as orc

pytestmark = pytest.mark.gpu

FIELD_RTOL = 1e-12  # GPU vs numpy FFT relative to the field max (second derivatives of a broadband q)


@pytest.fixture(scope="module")
def pv_series(tmp_path_factory, ctx):
    d = tmp_path_factory.mktemp("stored")
    nx = 512
    # 150 PDE steps: pv frames at steps 0, 50, 100, 150 (qgsw_raytrace.m:165-172)
    sw.qgsw_raytrace(nx, 0, 4.0, 10.0, 0.0, 0.2, 3.0, 1.0, out_dir=str(d), max_steps=150, r_drag=0.0, ctx=ctx)
    return d, nx


def test_pv_series_layout(pv_series):
    d, nx = pv_series
    assert sw.stored.frame_count(str(d / "pv"), nx) == 4
    t = sw.read_field(str(d / "pv_time"))
    assert t.shape == (1, 4) and t[0, 0] == 0.0 and np.all(np.diff(t[0]) > 0)
    q = sw.read_field(str(d / "pv"), nx, nx, 1, [3])
    np.testing.assert_array_equal(sw.read_frame(str(d / "pv"), nx, 3), q)


def test_set_field_q_is_g2k_then_grid_U(ctx, pv_series):
    d, nx = pv_series
    q = sw.read_frame(str(d / "pv"), nx, 2)
    f, Cg = 3.0, 1.0
    ctx.set_field_q(0, q, 2 * math.pi, f / Cg)
    a = ctx.get_field_grid(0)
    ctx.set_field_qk(1, ctx.g2k(q), nx, 2 * math.pi, f / Cg)
    np.testing.assert_array_equal(a, ctx.get_field_grid(1))
    kx_, ky_, K2 = orc.wavenumber_grids(nx)
    flow = orc.grid_U(orc.g2k(q), f / Cg, K2, kx_, ky_)
    for i, name in enumerate(orc.FIELD_ORDER):
        ref = np.asarray(flow[name]).ravel(order="F")
        assert np.abs(a[i] - ref).max() <= FIELD_RTOL * np.abs(ref).max(), name


def _packets(N, rng, L=2 * math.pi):
    x = L * rng.random((N, 2)) - L / 2
    i = np.arange(1, N + 1)
    wf = math.sqrt(15.0) * 3.0
    k = np.stack([wf * np.cos(2 * np.pi * i / N), wf * np.sin(2 * np.pi * i / N)], axis=1)
    return x, k


def test_trace_stored_matches_oracle_1e5(ctx, oracle_lib, pv_series):
    d, nx = pv_series
    f, Cg, nsub, L = 3.0, 1.0, 5, 2 * math.pi
    x0, k0 = _packets(100_000, np.random.default_rng(146))
    xs, ks, t_end = sw.trace_stored(str(d / "pv"), nx, x0, k0, f, Cg, nsub=nsub, ctx=ctx)
    t = sw.read_field(str(d / "pv_time"))[0]
    assert t_end == t[-1]
    # the oracle over the device's field bits, one interval per frame pair
    planes = []
    for fr in range(1, 5):
        ctx.set_field_q(0, sw.read_frame(str(d / "pv"), nx, fr), L, f / Cg)
        planes.append(ctx.get_field_grid(0).copy())
    x, k = x0, k0
    for i in range(3):
        h = (t[i + 1] - t[i]) / nsub
        x, k, _, _ = oracle_lib.leapfrog(planes[i], planes[i + 1], 0.5 / nsub, 1.0 / nsub, nx, nx, L / nx,
                                         orc.BUMP_QG, x, k, h, nsub, f, Cg ** 2)
    np.testing.assert_array_equal(xs, x)
    np.testing.assert_array_equal(ks, k)
    assert np.abs(xs - x0).max() > 1e-3  # the packets moved


def test_trace_stored_grouping_and_frames_written(ctx, pv_series, tmp_path):
    d, nx = pv_series
    x0, k0 = _packets(20_000, np.random.default_rng(5))
    a = sw.trace_stored(str(d / "pv"), nx, x0, k0, 3.0, 1.0, nsub=3, intervals_per_call=1, ctx=ctx,
                        out_dir=str(tmp_path))
    b = sw.trace_stored(str(d / "pv"), nx, x0, k0, 3.0, 1.0, nsub=3, intervals_per_call=4, ctx=ctx)
    np.testing.assert_array_equal(a[0], b[0])
    np.testing.assert_array_equal(a[1], b[1])
    xg = sw.read_field(str(tmp_path / "packet_x"), 20_000, 2, 1)
    assert xg.shape == (20_000, 2, 4)  # the first frame + one per interval
    L = 2 * math.pi
    np.testing.assert_array_equal(xg[:, :, -1], np.mod(a[0] + L / 2, L) - L / 2)


def test_trace_stored_two_layer_series(ctx, oracle_lib, tmp_path):
    """2-layer frames (nx x nx x 2): layer 1 is traced with the 2*nx y-period
    and k scaled by 2*pi/L (qg2layersw_raytrace.m:20-21,186-188)."""
    nx, L, f, Cg = 64, 20.0, 3.0, 1.0
    rng = np.random.default_rng(8)
    qs = []
    q1 = sw.qg.initial_q(nx, L, 0.2, f / Cg, 10, 30, rng, ndgrid=True)
    for i in range(3):
        q = np.stack([q1 * (1 + 0.1 * i), -q1], axis=2)
        sw.write_field(q, str(tmp_path / "pv"))
        sw.write_field(np.array([[0.5 * i]]), str(tmp_path / "pv_time"))
        qs.append(q)
    x0, k0 = _packets(3000, rng, L)
    ks_ = 2 * math.pi / L
    xs, kk, _ = sw.trace_stored(str(tmp_path / "pv"), nx, x0, k0, f, Cg, nlayers=2, L=L, shear=0.5, k_scale=ks_,
                                nsub=4, ctx=ctx)
    planes = []
    for q in qs:
        ctx.set_field_q(0, q[:, :, 0], L, f / Cg, 0.5, ks_, 2 * nx)
        planes.append(ctx.get_field_grid(0).copy())
    x, k = x0, k0
    for i in range(2):
        x, k, _, _ = oracle_lib.leapfrog(planes[i], planes[i + 1], 0.5 / 4, 1.0 / 4, nx, 2 * nx, L / nx,
                                         orc.BUMP_QG, x, k, 0.5 / 4, 4, f, Cg ** 2)
    np.testing.assert_array_equal(xs, x)
    np.testing.assert_array_equal(kk, k)
