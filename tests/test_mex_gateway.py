"""The MATLAB MEX gateway (matlab/swrt_mex.cpp) compiled against the test
mex.h shim (tests/mex_shim/, no MATLAB in the image) and driven through
ctypes: argument marshalling (column-major N x 2 arrays, interleaved complex,
structs, 3-D history frames), context handles (each SpectralSchemeGPU owns a
context, so two schemes never share fields — SpectralScheme.m:28-35), errors
raised through mexErrMsgIdAndTxt, and the drop-ins' index logic
(ode_symplectic_gpu.m's permute, SpectralSchemeGPU's U_field / GradU_field /
psi_field) against the oracle.  The MATLAB-side .m code is restated here in
numpy where a test needs it (cited line by line)."""
import ctypes
import os

import numpy as np
import pytest

from oracle import swrt_oracle as orc

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "build", "mex", "libswrt_mex_shim.so")
# GPU FFT vs numpy FFT, relative to the field's max: ~log2(n) eps times the
# ratio of the summed mode amplitudes to the max, which for the second
# derivatives of these broadband psi fields is ~10 (measured 1.1e-13 on v_x)
FIELD_RTOL = 1e-12
_vp = ctypes.c_void_p


class MexError(RuntimeError):
    pass


class Mex:
    """swrt_mex(...) as MATLAB would call it: numpy arrays <-> mxArrays."""

    def __init__(self):
        if not os.path.exists(SHIM):
            import __graft_entry__
            __graft_entry__.build()
        L = ctypes.CDLL(SHIM)
        L.shim_array.restype = _vp
        L.shim_array.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int, ctypes.POINTER(ctypes.c_size_t),
                                 ctypes.c_int]
        L.shim_string.restype = _vp
        L.shim_string.argtypes = [ctypes.c_char_p]
        L.shim_struct.restype = _vp
        L.shim_struct.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(_vp)]
        L.shim_free.argtypes = [_vp]
        L.shim_ndim.argtypes = [_vp]
        L.shim_dims.argtypes = [_vp, ctypes.POINTER(ctypes.c_size_t)]
        L.shim_is_complex.argtypes = [_vp]
        L.shim_ndata.restype = ctypes.c_size_t
        L.shim_ndata.argtypes = [_vp]
        L.shim_data.restype = ctypes.POINTER(ctypes.c_double)
        L.shim_data.argtypes = [_vp]
        L.shim_call.argtypes = [ctypes.c_int, ctypes.POINTER(_vp), ctypes.c_int, ctypes.POINTER(_vp),
                                ctypes.c_char_p, ctypes.c_int]
        self.L = L

    def _in(self, a):
        if isinstance(a, str):
            return self.L.shim_string(a.encode())
        if isinstance(a, dict):
            names = (ctypes.c_char_p * len(a))(*[k.encode() for k in a])
            vals = (_vp * len(a))(*[self._in(v) for v in a.values()])
            return self.L.shim_struct(len(a), names, vals)
        a = np.asarray(a)
        if a.ndim == 0:
            a = a.reshape(1, 1)
        cplx = np.iscomplexobj(a)
        flat = np.ascontiguousarray(np.ravel(a.astype(np.complex128 if cplx else np.float64), order="F"))
        data = flat.view(np.float64) if cplx else flat
        dims = (ctypes.c_size_t * a.ndim)(*a.shape)
        return self.L.shim_array(data.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.ndim, dims, int(cplx))

    def _out(self, p):
        nd = self.L.shim_ndim(p)
        dims = (ctypes.c_size_t * nd)()
        self.L.shim_dims(p, dims)
        n = self.L.shim_ndata(p)
        data = np.ctypeslib.as_array(self.L.shim_data(p), shape=(n,)).copy() if n else np.zeros(0)
        if self.L.shim_is_complex(p):
            data = data.view(np.complex128)
        out = data.reshape(tuple(dims), order="F")
        return out[0, 0] if out.shape == (1, 1) and not np.iscomplexobj(out) else out

    def __call__(self, cmd, *args, nlhs=1):
        prhs = [self._in(cmd)] + [self._in(a) for a in args]
        pr = (_vp * len(prhs))(*prhs)
        pl = (_vp * max(1, nlhs))()
        err = ctypes.create_string_buffer(1024)
        rc = self.L.shim_call(nlhs, pl, len(prhs), pr, err, 1024)
        for p in prhs:
            self.L.shim_free(p)
        outs = [self._out(p) if p else None for p in pl]
        for p in pl:
            if p:
                self.L.shim_free(p)
        if rc:
            raise MexError(err.value.decode())
        return outs[0] if nlhs <= 1 else outs


@pytest.fixture(scope="module")
def mex():
    return Mex()


def test_gateway_builds_and_exports_mexfunction():
    import subprocess
    if not os.path.exists(SHIM):
        import __graft_entry__
        __graft_entry__.build()
    syms = subprocess.run(["nm", "-D", "--defined-only", SHIM], capture_output=True, text=True, check=True).stdout
    assert " mexFunction" in syms


def test_gateway_argument_errors(mex):
    with pytest.raises(MexError, match="swrt:arg: first argument: command"):
        mex(3.0)
    with pytest.raises(MexError, match="second argument: the context handle"):
        mex("eval")
    with pytest.raises(MexError, match="invalid or closed context handle 7"):
        mex("eval", 7.0, np.zeros(3), np.zeros(3), 1.0, 0.0, 1e-13)
    with pytest.raises(MexError, match="invalid or closed context handle 1.5"):
        mex("qg_max_speed", 1.5)


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present")
def test_create_without_gpu_raises(mex):
    with pytest.raises(MexError, match="swrt:create: swrt_create failed"):
        mex("create", 0.0)


def _psi(nx, seed):
    X, Y = np.meshgrid(np.arange(nx) * (2 * np.pi / nx), np.arange(nx) * (2 * np.pi / nx), indexing="ij")
    rng = np.random.default_rng(seed)
    psi = np.zeros((nx, nx))
    for _ in range(12):
        kx, ky = rng.integers(-6, 7, 2)
        psi += 0.05 * rng.normal() / (1 + kx * kx + ky * ky) * np.cos(kx * X + ky * Y + rng.uniform(0, 6))
    return psi


def _scheme_gpu(mex, psi, L=2 * np.pi):
    """SpectralSchemeGPU.m constructor: its own context, field in slot 0,
    psi_field = k2g(g2k(psi)) from the device (SpectralScheme.m:28)."""
    h = mex("create", 0.0)
    mex("set_field_psi", h, 0.0, psi, L)
    return h


@pytest.mark.gpu
def test_two_schemes_are_independent_and_match_oracle(mex, oracle_lib):
    nx, L = 64, 2 * np.pi
    psi1, psi2 = _psi(nx, 1), _psi(nx, 2)
    rng = np.random.default_rng(3)
    x = rng.uniform(-L, L, 500)
    y = rng.uniform(-L, L, 500)
    h1 = _scheme_gpu(mex, psi1)
    before = mex("eval", h1, x, y, 1.0, 0.0, orc.BUMP_SW)
    h2 = _scheme_gpu(mex, psi2)
    after = mex("eval", h1, x, y, 1.0, 0.0, orc.BUMP_SW)
    other = mex("eval", h2, x, y, 1.0, 0.0, orc.BUMP_SW)
    assert h1 != h2 and before.shape == (500, 6)
    np.testing.assert_array_equal(before, after)  # the second scheme did not touch the first
    assert np.abs(other - before).max() > 1e-3
    for h, psi, got in ((h1, psi1, after), (h2, psi2, other)):
        F = mex("get_fields", h, 0.0, float(nx))  # SpectralSchemeGPU.get.U_field / get.GradU_field
        assert F.shape == (nx, nx, 6)
        ref = orc.SpectralSchemeOracle(L, nx, psi)
        for i, name in enumerate(orc.FIELD_ORDER):
            d = np.abs(F[:, :, i] - ref.fields[name]).max() / np.abs(ref.fields[name]).max()
            assert d < FIELD_RTOL, name
        pf = mex("get_psi", h, 0.0, float(nx))  # SpectralSchemeGPU.psi_field
        assert np.abs(pf - ref.psi_field).max() < FIELD_RTOL * np.abs(ref.psi_field).max()
        # eval is the oracle's arithmetic on the device's fields, bit for bit
        planes = np.ascontiguousarray(np.stack([F[:, :, i].ravel(order="F") for i in range(6)]))
        o = oracle_lib.eval6(planes, None, 0.0, nx, nx, L / nx, orc.BUMP_SW, x, y)
        np.testing.assert_array_equal(got, o.T)
    mex("destroy", h2)
    with pytest.raises(MexError, match="invalid or closed context handle"):
        mex("eval", h2, x, y, 1.0, 0.0, orc.BUMP_SW)
    np.testing.assert_array_equal(mex("eval", h1, x, y, 1.0, 0.0, orc.BUMP_SW), before)
    mex("destroy", h1)


@pytest.mark.gpu
def test_ode_symplectic_gpu_layout_matches_ode_symplectic(mex):
    """ode_symplectic_gpu.m:13-25 (Nsteps x 2 x P from the gateway's P x 2 x
    (Nsteps-1) history by permute([3 2 1])) equals ode_symplectic.m run on
    the same scheme fields, bit for bit."""
    nx, L, P = 64, 2 * np.pi, 37
    psi = _psi(nx, 4)
    h = _scheme_gpu(mex, psi)
    rng = np.random.default_rng(5)
    x0 = (L * rng.random((1, 2, P)) - L / 2)
    th = 2 * np.pi * np.arange(1, P + 1) / P
    k0 = 3.0 * np.stack([np.cos(th), np.sin(th)])[None]
    dt, T, f, gH = 0.02, 0.02 * 23.5, 3.0, 1.0
    # --- ode_symplectic_gpu.m ---
    Nsteps = int(np.floor(T / dt))
    X0 = np.reshape(x0, (2, P), order="F").T  # reshape(x0, 2, P)'
    K0 = np.reshape(k0, (2, P), order="F").T
    _, _, hx, hk = mex("leapfrog", h, X0, K0, dt, float(Nsteps - 1), f, gH, 1.0, 0.0, 0.0, orc.BUMP_SW, 1.0,
                       nlhs=4)
    assert hx.shape == (P, 2, Nsteps - 1)
    xg = np.zeros((Nsteps, 2, P))
    kg = np.zeros((Nsteps, 2, P))
    xg[0], kg[0] = x0[0], k0[0]
    xg[1:] = np.transpose(hx, (2, 1, 0))  # permute(hx, [3 2 1])
    kg[1:] = np.transpose(hk, (2, 1, 0))
    # --- ode_symplectic.m on the device's fields ---
    F = mex("get_fields", h, 0.0, float(nx))
    sch = orc.SpectralSchemeOracle(L, nx, psi)
    sch.fields = {name: F[:, :, i] for i, name in enumerate(orc.FIELD_ORDER)}
    xo, ko, t = orc.ode_symplectic(x0, k0, dt, T, f, gH, sch)
    np.testing.assert_array_equal(xg, xo)
    np.testing.assert_array_equal(kg, ko)
    mex("destroy", h)


@pytest.mark.gpu
def test_spectral_and_qg_commands(mex, ctx):
    """g2k / k2g (interleaved complex both ways) and the qg_* commands with a
    params struct: the same device code as the Python front end, so the same
    bits as swraytracing_amd's QGModel."""
    import swraytracing_amd as sw
    nx = 64
    h = mex("create", 0.0)
    g = _psi(nx, 8)
    fk = mex("g2k", h, g)
    assert fk.shape == (nx - 1, nx // 2) and np.iscomplexobj(fk)
    np.testing.assert_array_equal(fk, ctx.g2k(g))
    assert np.abs(fk - orc.g2k(g)).max() < FIELD_RTOL * np.abs(orc.g2k(g)).max()
    np.testing.assert_array_equal(mex("k2g", h, fk), ctx.k2g(fk))
    qk0 = np.stack([fk, -fk], axis=2)
    p = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=20.0, ctx=ctx).params
    params = {"nlayers": 2.0, "filter": float(p.filter), "L": p.L, "K_d2": p.K_d2, "beta": p.beta, "r_drag": p.r_drag,
              "force_strength": p.force_strength, "f": p.f, "Cg": p.Cg, "shear": p.shear, "nu": p.nu,
              "hyper_order": p.hyper_order, "r": p.r}
    mex("qg_init", h, params, qk0)
    U0 = mex("qg_max_speed", h)
    dt = 0.25 * (20.0 / nx) / U0
    mex("qg_step", h, dt, 5.0)
    qk, t, steps = mex("qg_get", h, float(nx), 2.0, nlhs=3)
    m = sw.QGModel.two_layer(qk0, nx, 3.0, 1.0, L=20.0, ctx=ctx)
    assert m.max_speed() == U0
    m.step(dt, 5)
    np.testing.assert_array_equal(qk, m.qk)
    assert steps == 5 and t == m.t
    q = mex("qg_get_q", h, float(nx), 2.0)
    np.testing.assert_array_equal(q, m.q())
    mex("qg_snapshot", h, 0.0, 0.0, 0.0, float(2 * nx))
    assert mex("field_div_free", h, 0.0) == 1.0
    mex("destroy", h)


def _ode23_packets_gpu_m(mex, hctx, tspan, tmax, f, Cg, nslots):
    """matlab/ode23_packets_gpu.m line for line (MATLAB eps(t) = np.spacing)."""
    rtol, atol, bump = max(1e-3, 100 * np.finfo(float).eps), 1e-6, 1e-10
    thr, pw = atol / rtol, 1.0 / 3.0
    t0, tfinal = tspan
    tdir = np.sign(tfinal - t0)
    htspan = abs(tfinal - t0)
    hmax = 0.1 * htspan
    t = t0
    rh = mex("ode23_f1", hctx, t, tmax, f, Cg, nslots, thr, bump) / (0.8 * rtol ** pw)
    absh = min(hmax, htspan)
    if absh * rh > 1:
        absh = 1 / rh
    absh = max(absh, 16 * np.spacing(t))
    acc, done = [t], False
    while not done:
        hmin = 16 * np.spacing(t)
        absh = min(hmax, max(hmin, absh))
        h = tdir * absh
        if 1.1 * absh >= abs(tfinal - t):
            h = tfinal - t
            absh = abs(h)
            done = True
        nofailed = True
        while True:
            tnew = t + h
            if done:
                tnew = tfinal
            err = absh * mex("ode23_attempt", hctx, t, h, tnew, tmax, f, Cg, nslots, thr, bump)
            h = tnew - t
            if err > rtol:
                if nofailed:
                    nofailed = False
                    absh = max(hmin, absh * max(0.5, 0.8 * (rtol / err) ** pw))
                else:
                    absh = max(hmin, 0.5 * absh)
                h = tdir * absh
                done = False
            else:
                break
        mex("ode23_accept", hctx)
        t = tnew
        acc.append(t)
        if done:
            break
        if nofailed:
            temp = 1.25 * (err / rtol) ** pw
            absh = absh / temp if temp > 0.2 else 5.0 * absh
    return np.array(acc)


@pytest.mark.gpu
def test_ode23_packets_gpu_m_matches_python_controller(mex, ctx, qg_case):
    """ode23_packets_gpu.m over the gateway (fields through set_field_grid:
    six nx x nx matrices, L, ny_period; packets through packets_set/get) gives
    the accepted times and packets of the Python controller (integrate.
    ode23_packets) on the same device code, bit for bit."""
    import swraytracing_amd as sw
    c = qg_case
    nx, L = c["nx"], c["L"]
    fl1 = c["flow"]
    fl2 = {n: np.asarray(v) * 1.07 for n, v in fl1.items()}
    dt = c["dt"] * 20
    h = mex("create", 0.0)
    for slot, fl in ((0.0, fl1), (1.0, fl2)):
        mex("set_field_grid", h, slot, *[np.asarray(fl[n]) for n in orc.FIELD_ORDER], L, float(nx))
    mex("packets_set", h, c["x"], c["k"])
    tm = _ode23_packets_gpu_m(mex, h, (0.0, dt), dt, c["f"], c["Cg"], 2.0)
    xm, km = mex("packets_get", h, nlhs=2)
    mex("destroy", h)
    planes = lambda fl: np.ascontiguousarray(np.stack([np.asarray(fl[n]).ravel(order="F") for n in orc.FIELD_ORDER]))
    ctx.set_field_grid(0, planes(fl1), nx, L, nx)
    ctx.set_field_grid(1, planes(fl2), nx, L, nx)
    ctx.packets_set(c["x"], c["k"])
    tp = sw.integrate.ode23_packets(ctx, (0.0, dt), dt, c["f"], c["Cg"], 2, bump=1e-10)
    xp, kp = ctx.packets_get()
    np.testing.assert_array_equal(tm, tp)
    np.testing.assert_array_equal(xm, xp)
    np.testing.assert_array_equal(km, kp)
    assert len(tm) > 2


class _SwrtContext:
    """matlab/SwrtContext.m restated (a MATLAB handle object: delete runs when
    its last reference goes, release() closes it for every holder)."""

    def __init__(self, mex, device=0.0):
        self.mex = mex
        self.h = mex("create", device)

    def id(self):
        if self.h == 0:
            raise MexError("swrt:state: closed context")
        return self.h

    def release(self):
        if self.h != 0:
            self.mex("destroy", self.h)
            self.h = 0

    def __del__(self):
        self.release()


@pytest.mark.gpu
def test_scheme_contexts_freed_with_last_reference(mex):
    """One SpectralSchemeGPU per snapshot (50 of them, each dropped after
    use) keeps at most one context open; value copies share one SwrtContext
    (SpectralSchemeGPU.m ctx), which stays open until the last copy goes."""
    import gc
    nx = 64
    base = mex("live")
    peak = 0
    for i in range(50):
        ctx = _SwrtContext(mex)                      # SpectralSchemeGPU ctor: obj.ctx = SwrtContext(0)
        mex("set_field_psi", ctx.id(), 0.0, _psi(nx, i), 2 * np.pi)
        peak = max(peak, mex("live") - base)
        del ctx
        gc.collect()
    assert peak == 1 and mex("live") == base
    a = _SwrtContext(mex)
    copy = a                                         # s2 = s1: a value copy holds the same handle object
    mex("set_field_psi", a.id(), 0.0, _psi(nx, 1), 2 * np.pi)
    del a
    gc.collect()
    assert mex("live") == base + 1                   # the copy keeps it open
    F = mex("get_fields", copy.id(), 0.0, float(nx))
    assert F.shape == (nx, nx, 6)
    with pytest.raises(MexError, match=r"holds a 64\^2 grid, not 32\^2"):
        mex("get_fields", copy.id(), 0.0, 32.0)      # the library's size, never the caller's
    h = copy.h
    copy.release()                                   # release(scheme): closed for every copy
    assert mex("live") == base
    with pytest.raises(MexError, match="closed context"):
        copy.id()
    with pytest.raises(MexError, match="invalid or closed context handle"):
        mex("get_fields", h, 0.0, float(nx))


@pytest.mark.gpu
def test_trace_stored_gpu_m_matches_trace_stored(mex, ctx, tmp_path):
    """matlab/trace_stored_gpu.m over the gateway (frames by read_field ->
    set_field_q, intervals by advance_intervals at nsub substeps, four per
    call, swap_slots between calls) gives the packets of the Python twin
    swraytracing_amd.trace_stored on the same PV series, bit for bit."""
    import swraytracing_amd as sw
    nx, L, f, Cg, nsub = 64, 2 * np.pi, 3.0, 1.0, 5
    rng = np.random.default_rng(21)
    q1 = sw.qg.initial_q(nx, L, 0.2, f / Cg, 3, 8, rng)
    for i in range(6):  # six frames: one call of four intervals, one of one
        sw.write_field(q1 * (1 + 0.05 * i), str(tmp_path / "pv"))
        sw.write_field(np.array([[0.3 * i + 0.01 * i * i]]), str(tmp_path / "pv_time"))
    x0 = L * rng.random((3000, 2)) - L / 2
    k0 = rng.normal(0.0, 5.0, (3000, 2))
    xs, ks, t_end = sw.trace_stored(str(tmp_path / "pv"), nx, x0, k0, f, Cg, nsub=nsub, ctx=ctx)
    # trace_stored_gpu.m line by line (MATLAB's 1-based frames / times)
    times = sw.read_field(str(tmp_path / "pv_time"))[0]
    frames = list(range(1, 7))
    h = mex("create", 0.0)
    try:
        mex("packets_set", h, x0, k0)
        mex("set_locality", h, 4.0 * nsub, 0.0)

        def load_frame(slot, fr):
            q = sw.read_frame(str(tmp_path / "pv"), nx, fr)
            mex("set_field_q", h, float(slot), q, L, f / Cg, 0.0, 1.0, float(nx))

        load_frame(0, frames[0])
        i = 2
        while i <= len(frames):
            g = min(4, len(frames) - i + 1)
            for j in range(g):
                load_frame(1 + j, frames[i + j - 1])
            mex("advance_intervals", h, np.diff(times[i - 2:i + g - 1]) / nsub, float(nsub), f, Cg ** 2,
                0.5 / nsub, 1.0 / nsub, 1e-10)
            mex("swap_slots", h, 0.0, float(g))
            i += g
        xm, km = mex("packets_get", h, nlhs=2)
    finally:
        mex("destroy", h)
    assert t_end == times[-1]
    np.testing.assert_array_equal(np.asarray(xm).view(np.uint64), np.ascontiguousarray(xs).view(np.uint64))
    np.testing.assert_array_equal(np.asarray(km).view(np.uint64), np.ascontiguousarray(ks).view(np.uint64))
    assert np.abs(xs - x0).max() > 1e-3  # the packets moved
