"""Background-flow schemes: the reference's L2 boundary API on the GPU.

Mirrors RaytracingScheme.m (abstract streamfunction/U/grad_U + concrete
grad_U_times_k/vorticity/strain/okuboWeiss) and SpectralScheme.m (spectral
streamfunction -> gridded U, grad U, 6x6 Lagrange interpolation), plus the
qg drivers' grid_U / interpolate_U pair (qg_flow_ray_trace/grid_U.m,
interpolate_U.m).  All arithmetic runs in libswrt (HIP, gfx950).
"""
from __future__ import annotations

import abc
import math

import numpy as np

from ._lib import Context

BUMP_QG = 1e-10  # qg_flow_ray_trace/interpolate.m:13 (qg drivers, interpolate_U)
BUMP_SW = 1e-13  # ray_trace_sw/interpolate.m:13 (SpectralScheme path, addpath order)

FIELD_ORDER = ("u", "v", "ux", "uy", "vx", "vy")

_default_ctx = {}


def default_context(device: int = 0) -> Context:
    """One shared context per device for the functional API."""
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def _split_xy(x):
    """x: M x 2 x P (MATLAB 3-D) or N x 2 -> flat xx, yy (column-major order)."""
    x = np.asarray(x, dtype=np.float64)
    xx = np.ravel(x[:, 0, ...], order="F")
    yy = np.ravel(x[:, 1, ...], order="F")
    return x, xx, yy


class RaytracingScheme(abc.ABC):
    """RaytracingScheme.m:1-33."""

    @abc.abstractmethod
    def streamfunction(self, x, y, t=0.0):
        ...

    @abc.abstractmethod
    def U(self, x, t=0.0):
        ...

    @abc.abstractmethod
    def grad_U(self, x, t=0.0):
        ...

    def grad_U_times_k(self, x, k, t=0.0):
        """RaytracingScheme.m:9-16: [u_x k + v_x l, u_y k + v_y l], size(k)."""
        nab = self.grad_U(x, t)
        k = np.asarray(k, dtype=np.float64)
        kk = np.ravel(k[:, 0, ...], order="F")
        ll = np.ravel(k[:, 1, ...], order="F")
        out = np.zeros_like(k)
        shp = k[:, 0, ...].shape
        out[:, 0, ...] = np.reshape(nab["u_x"] * kk + nab["v_x"] * ll, shp, order="F")
        out[:, 1, ...] = np.reshape(nab["u_y"] * kk + nab["v_y"] * ll, shp, order="F")
        return out

    def vorticity(self, x, t=0.0):
        nab = self.grad_U(x, t)
        return nab["v_x"] - nab["u_y"]  # RaytracingScheme.m:18-21

    def strain(self, x, t=0.0):
        nab = self.grad_U(x, t)  # RaytracingScheme.m:23-26
        return np.sqrt((nab["u_x"] - nab["v_y"]) ** 2 + (nab["v_x"] + nab["u_y"]) ** 2)

    def okuboWeiss(self, x, t=0.0):
        """RaytracingScheme.m:28-31 (the reference passes an undefined `k` to
        grad_U; the evident intent, grad_U(x, t), is implemented)."""
        nab = self.grad_U(x, t)
        return nab["v_y"] ** 2 + nab["v_x"] * nab["u_y"]


class SpectralScheme(RaytracingScheme):
    """SpectralScheme(L, nx, psi_field) (SpectralScheme.m:1-70) on the GPU.

    The constructor runs g2k, the six derivative spectra and k2g on the device
    (swrt_set_field_psi); U / grad_U interpolate there (swrt_eval).  Integer
    wavenumbers are assumed regardless of L, exactly as the reference does."""

    def __init__(self, L, nx, psi_field, device: int = 0, bump: float = BUMP_SW, ctx: Context | None = None):
        self.L = float(L)
        self.nx = int(nx)
        self.bump = bump
        self.ctx = ctx if ctx is not None else Context(device)
        psi = np.asarray(psi_field, dtype=np.float64)
        if psi.shape != (self.nx, self.nx):
            raise ValueError(f"psi_field must be {nx} x {nx}, got {psi.shape}")
        self.ctx.set_field_psi(0, psi, self.nx, self.L)
        self._psi = None
        self._planes = None

    # reference properties (downloaded lazily; the device copy is authoritative)
    @property
    def psi_field(self):
        if self._psi is None:
            self._psi = self.ctx.get_psi_grid(0, self.nx)
        return self._psi

    def _fields(self):
        if self._planes is None:
            p = self.ctx.get_field_grid(0, self.nx)
            self._planes = {n: p[i].reshape((self.nx, self.nx), order="F") for i, n in enumerate(FIELD_ORDER)}
        return self._planes

    @property
    def U_field(self):
        f = self._fields()
        return {"u": f["u"], "v": f["v"]}

    @property
    def GradU_field(self):
        f = self._fields()
        return {"u_x": f["ux"], "u_y": f["uy"], "v_x": f["vx"], "v_y": f["vy"]}

    @property
    def dx(self):
        return self.L / self.nx  # SpectralScheme.m:46

    def streamfunction(self, x, y, t=0.0):
        """SpectralScheme.m:38-43."""
        x = np.asarray(x, dtype=np.float64)
        out = self.ctx.interpolate(x, y, self.psi_field, self.dx, self.dx, self.bump)
        return out.reshape(x.shape)

    def _eval(self, x):
        x, xx, yy = _split_xy(x)
        return x, self.ctx.eval(xx, yy, nslots=1, bump=self.bump)

    def U(self, x, t=0.0):
        """SpectralScheme.m:45-54: returns size(x)."""
        x, I = self._eval(x)
        u = np.zeros_like(x)
        shp = x[:, 0, ...].shape
        u[:, 0, ...] = np.reshape(I[0], shp, order="F")
        u[:, 1, ...] = np.reshape(I[1], shp, order="F")
        return u

    def grad_U(self, x, t=0.0):
        """SpectralScheme.m:56-68: struct of numel(x)/2 columns."""
        _, I = self._eval(x)
        return {"u_x": I[2], "u_y": I[3], "v_x": I[4], "v_y": I[5]}


class SnapshotPairScheme(RaytracingScheme):
    """Two gridded snapshots blended in time (interpolate_U.m:1-24): the
    background the qg drivers feed ode23 (qgsw_raytrace.m:141-143).  Scheme
    time t maps to alpha = t / tmax (generate_raytracing_ode, :258-261)."""

    def __init__(self, flow1, flow2, L, tmax=1.0, ny_period=0, device: int = 0, bump: float = BUMP_QG,
                 ctx: Context | None = None):
        self.ctx = ctx if ctx is not None else Context(device)
        self.L = float(L)
        self.tmax = float(tmax)
        self.bump = bump
        u = np.asarray(flow1["u"])
        self.nx = u.shape[0]
        self.ny_period = ny_period or (self.nx * (u.shape[2] if u.ndim == 3 else 1))
        for slot, fl in enumerate((flow1, flow2)):
            self.ctx.set_field_grid(slot, flow_planes(fl), self.nx, self.L, self.ny_period)

    @property
    def dx(self):
        return self.L / self.nx

    def streamfunction(self, x, y, t=0.0):  # pragma: no cover - grid_U keeps no psi
        raise NotImplementedError("grid_U snapshots carry no streamfunction")

    def _eval(self, x, t):
        x, xx, yy = _split_xy(x)
        return x, self.ctx.eval(xx, yy, nslots=2, alpha=t / self.tmax, bump=self.bump)

    def U(self, x, t=0.0):
        x, I = self._eval(x, t)
        u = np.zeros_like(x)
        shp = x[:, 0, ...].shape
        u[:, 0, ...] = np.reshape(I[0], shp, order="F")
        u[:, 1, ...] = np.reshape(I[1], shp, order="F")
        return u

    def grad_U(self, x, t=0.0):
        _, I = self._eval(x, t)
        return {"u_x": I[2], "u_y": I[3], "v_x": I[4], "v_y": I[5]}


class DifferenceScheme(RaytracingScheme):
    """DifferenceScheme.m:1-48: centred differences of an analytic psi(x,y,t)
    callback with h = eps^(1/3).  Host-side (an arbitrary Python callable);
    not part of the GPU hot path."""

    def __init__(self, stream):
        self.h = np.finfo(float).eps ** (1.0 / 3.0)
        self.psi = stream

    def streamfunction(self, x, y, t=0.0):
        return self.psi(x, y, t)

    def U(self, x, t=0.0):
        x = np.asarray(x, dtype=np.float64)
        xx = x[:, 0:1, ...]
        yy = x[:, 1:2, ...]
        h = self.h
        u = np.zeros_like(x)
        u[:, 1:2, ...] = (self.psi(xx + h / 2, yy, t) - self.psi(xx - h / 2, yy, t)) / h
        u[:, 0:1, ...] = -(self.psi(xx, yy + h / 2, t) - self.psi(xx, yy - h / 2, t)) / h
        return u

    def grad_U(self, x, t=0.0):
        x = np.asarray(x, dtype=np.float64)
        xx = np.ravel(x[:, 0, ...], order="F")
        yy = np.ravel(x[:, 1, ...], order="F")
        h = self.h
        p = self.psi
        v_x = (p(xx + h, yy, t) - 2 * p(xx, yy, t) + p(xx - h, yy, t)) / h / h
        u_y = -(p(xx, yy + h, t) - 2 * p(xx, yy, t) + p(xx, yy - h, t)) / h / h
        v_y = (p(xx + h / 2, yy + h / 2, t) + p(xx - h / 2, yy - h / 2, t)
               - p(xx - h / 2, yy + h / 2, t) - p(xx + h / 2, yy - h / 2, t)) / h / h
        return {"u_x": -v_y, "u_y": u_y, "v_x": v_x, "v_y": v_y}


# ----------------------------------------------------------------------------
# Functional API of qg_flow_ray_trace/ (GPU)
# ----------------------------------------------------------------------------
def flow_planes(flow):
    """grid_U struct (u, v, ux, uy, vx, vy; nx x nx or nx x nx x nz, layer 1
    read) -> 6 x nx*nx column-major planes."""
    planes = []
    for n in FIELD_ORDER:
        a = np.asarray(flow[n], dtype=np.float64)
        if a.ndim == 3:
            a = a[:, :, 0]
        planes.append(a.ravel(order="F"))
    return np.ascontiguousarray(np.stack(planes))


def interpolate(x, y, F, dx, dy, bump=BUMP_QG, ctx: Context | None = None):
    """interpolate.m:1-50 on the GPU (bump 1e-10 = qg_flow_ray_trace copy)."""
    return (ctx or default_context()).interpolate(x, y, F, dx, dy, bump)


def interpolate_U(flow1, flow2, alpha, x, h, bump=BUMP_QG, ctx: Context | None = None):
    """interpolate_U.m:1-24 on the GPU.  x: N x 2.  Returns U (N x 2), nablaU."""
    ctx = ctx or default_context()
    u = np.asarray(flow1["u"])
    nx = u.shape[0]
    nyp = nx * (u.shape[2] if u.ndim == 3 else 1)
    L = h * nx
    ctx.set_field_grid(0, flow_planes(flow1), nx, L, nyp)
    ctx.set_field_grid(1, flow_planes(flow2), nx, L, nyp)
    x = np.asarray(x, dtype=np.float64)
    I = ctx.eval(x[:, 0], x[:, 1], nslots=2, alpha=alpha, bump=bump)
    U = np.stack([I[0], I[1]], axis=1)
    return U, {"u_x": I[2], "u_y": I[3], "v_x": I[4], "v_y": I[5]}


def g2k(fg, ctx: Context | None = None):
    """g2k.m on the GPU."""
    return (ctx or default_context()).g2k(fg)


def k2g(fk, ctx: Context | None = None):
    """k2g.m (+fulspec.m) on the GPU; real part."""
    return (ctx or default_context()).k2g(fk)


def _k_scale_of(kx_, ky_, nx):
    kmax = nx // 2 - 1
    kx_ = np.asarray(kx_, dtype=np.float64)
    s = kx_[kmax + 1, 0]  # kx = +1 row
    ints_x, ints_y = np.meshgrid(np.arange(-kmax, kmax + 1.0), np.arange(0, kmax + 1.0), indexing="ij")
    if not (np.allclose(kx_, ints_x * s, rtol=1e-14, atol=0) and
            np.allclose(np.asarray(ky_), ints_y * s, rtol=1e-14, atol=0)):
        raise ValueError("kx_, ky_ must be ndgrid(-kmax:kmax, 0:kmax) times a common scale")
    return float(s)


def grid_U(qk, K_d2, K2, kx_, ky_, shear_strength=0.0, ctx: Context | None = None):
    """grid_U.m:1-18 on the GPU (per layer for a 3-D qk, apply_3d.m).

    K2 must be kx_.^2 + ky_.^2 (as every call site builds it)."""
    ctx = ctx or default_context()
    qk = np.asarray(qk, dtype=np.complex128)
    nx = qk.shape[0] + 1
    s = _k_scale_of(kx_, ky_, nx)
    layers = [qk] if qk.ndim == 2 else [qk[:, :, i] for i in range(qk.shape[2])]
    out = {n: [] for n in FIELD_ORDER}
    for q in layers:
        ctx.set_field_qk(0, q, nx, 2 * math.pi, K_d2, shear_strength, s, 0)
        p = ctx.get_field_grid(0, nx)
        for i, n in enumerate(FIELD_ORDER):
            out[n].append(p[i].reshape((nx, nx), order="F"))
    if qk.ndim == 2:
        return {n: v[0] for n, v in out.items()}
    return {n: np.stack(v, axis=2) for n, v in out.items()}


class FourierScheme(RaytracingScheme):
    """Exact spectral evaluation of the background (no grid, no interpolation):
    the evaluator of scratch/fourier_interpolate_test.m:92-136, generalised to
    any dense mode grid, on the GPU (swrt_spectral_*).  Construct from a g2k
    half-plane streamfunction spectrum or from the scratch test's amp/phase."""

    def __init__(self, C, kx0, ky0, s, precision=64, device: int = 0, ctx: Context | None = None):
        self.ctx = ctx if ctx is not None else Context(device)
        self.precision = precision
        self.ctx.spectral_set_modes(C, kx0, ky0, s)

    @classmethod
    def from_halfplane(cls, psik, k_scale=1.0, **kw):
        psik = np.asarray(psik, dtype=np.complex128)
        kmax = psik.shape[1] - 1
        C = 2 * psik
        C[:kmax, 0] = 0
        C[kmax, 0] = psik[kmax, 0].real
        return cls(C, -kmax, 0, k_scale, **kw)

    @classmethod
    def from_amp_phase(cls, amp, phase, n, **kw):
        return cls(np.asarray(amp) * np.exp(1j * np.asarray(phase)), -n, -n, 1.0, **kw)

    def streamfunction(self, x, y, t=0.0):  # pragma: no cover - not needed by the integrators
        raise NotImplementedError

    def _eval(self, x):
        x, xx, yy = _split_xy(x)
        return x, self.ctx.spectral_eval(xx, yy, self.precision)

    def U(self, x, t=0.0):
        x, I = self._eval(x)
        u = np.zeros_like(x)
        shp = x[:, 0, ...].shape
        u[:, 0, ...] = np.reshape(I[0], shp, order="F")
        u[:, 1, ...] = np.reshape(I[1], shp, order="F")
        return u

    def grad_U(self, x, t=0.0):
        _, I = self._eval(x)
        return {"u_x": I[2], "u_y": I[3], "v_x": I[4], "v_y": I[5]}

    def leapfrog(self, x, k, dt, nsteps, f, gH):
        """Fused device leapfrog with the exact kick (x, k: N x 2)."""
        return self.ctx.spectral_leapfrog(x, k, dt, nsteps, f, gH, self.precision)
