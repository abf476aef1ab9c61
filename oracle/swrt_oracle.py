"""CPU oracle for the qg_flow_ray_trace hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain-numpy restatement of the MATLAB reference
(ndefilippis/SWRaytracing) for the wave-packet ray-tracing hot loop.  It exists
to *check* the HIP product path; it is never imported by the product package
(`swraytracing_amd/`), only by `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py`.

Parity status: the reference is MATLAB and cannot run
in this container (no MATLAB/Octave), and it ships no numeric golden vectors,
fixtures or tests.  This restatement is therefore pinned by analytic known
answers only (zero background flow, single Fourier mode, the closed-form
random Fourier field of scratch/fourier_interpolate_test.m, k2g(g2k(f)) == f,
Lagrange-weight identities) — "parity pinned to analytic KATs; no
reference-produced vectors exist".

Every function follows the cited .m file line by line, including operation
order (so that the same IEEE-754 double operations happen in the same order as
in MATLAB's scalar loops), MATLAB `mod` semantics and the 1-based index maths
(done here 0-based with identical results).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

IORD = 2  # interpolate.m:12 — 6x6 Lagrange stencil
BUMP_QG = 1e-10  # qg_flow_ray_trace/interpolate.m:13
BUMP_SW = 1e-13  # ray_trace_sw/interpolate.m:13 (SpectralScheme path via addpath, SpectralScheme.m:7-8)


# ----------------------------------------------------------------------------
# MATLAB primitives
# ----------------------------------------------------------------------------
def matlab_mod(a, m):
    """MATLAB mod(a, m) = a - floor(a./m).*m for m > 0 (documented definition).

    With integer m (always the case here: m = nx or nlayers*nx) MATLAB's
    round-off compensation for non-integer divisors does not apply.
    """
    a = np.asarray(a, dtype=np.float64)
    return a - np.floor(a / m) * m


# ----------------------------------------------------------------------------
# L1 spectral utilities — qg_flow_ray_trace/{g2k,k2g,fulspec,apply_3d}.m
# ----------------------------------------------------------------------------
def g2k(fg):
    """g2k.m:5-9: fk = fftshift(fft2(fg))/nx^2, rows 2:end, cols kmax+2:end."""
    fg = np.asarray(fg, dtype=np.float64)
    nx = fg.shape[0]
    kmax = nx // 2 - 1
    fkt = np.fft.fftshift(np.fft.fft2(fg)) / nx**2
    return fkt[1:, kmax + 1:].copy()


def fulspec(fk):
    """fulspec.m:10-19: Hermitian completion of the upper-half spectrum."""
    fk = np.asarray(fk, dtype=np.complex128)
    nkx, nky = fk.shape
    nx = nkx + 1
    kmax = nky - 1
    fkf = np.zeros((nx, nx), dtype=np.complex128)
    fup = fk.copy()
    # fup(kmax:-1:1,1) = conj(fup(kmax+2:nkx,1))      (fulspec.m:16)
    fup[kmax - 1::-1, 0] = np.conj(fup[kmax + 1:nkx, 0])
    # fdn = conj(fup(nkx:-1:1,nky:-1:2))              (fulspec.m:17)
    fdn = np.conj(fup[::-1, nky - 1:0:-1])
    fkf[1:nx, nky:nx] = fup  # fulspec.m:18
    fkf[1:nx, 1:nky] = fdn  # fulspec.m:19
    return fkf


def k2g(fk):
    """k2g.m:5-6: fg = nx^2*ifft2(ifftshift(fulspec(fk))).

    The completed spectrum is Hermitian except possibly an imaginary DC part;
    MATLAB would then return a complex array whose real part is what every
    consumer (interpolate) effectively uses.  We return the real part.
    """
    fk = np.asarray(fk, dtype=np.complex128)
    nx = fk.shape[0] + 1
    fg = nx**2 * np.fft.ifft2(np.fft.ifftshift(fulspec(fk)))
    return np.ascontiguousarray(fg.real)


def apply_3d(x, f):
    """apply_3d.m:1-7 — apply f per layer along the 3rd dimension."""
    x = np.asarray(x)
    if x.ndim == 2:
        return f(x)
    first = f(x[:, :, 0])
    y = np.zeros(first.shape + (x.shape[2],), dtype=first.dtype)
    for i in range(x.shape[2]):
        y[:, :, i] = f(x[:, :, i])
    return y


def wavenumber_grids(nx, L=2 * math.pi, scale=False):
    """[kx_,ky_] = ndgrid(-kmax:kmax, 0:kmax) (qgsw_raytrace.m:18-20).

    With scale=True multiply by 2*pi/L (qg2layersw_raytrace.m:19-22).
    """
    kmax = nx // 2 - 1
    kx_, ky_ = np.meshgrid(np.arange(-kmax, kmax + 1, dtype=np.float64),
                           np.arange(0, kmax + 1, dtype=np.float64), indexing="ij")
    if scale:
        kx_ = kx_ * (2 * math.pi / L)
        ky_ = ky_ * (2 * math.pi / L)
    K2 = kx_**2 + ky_**2
    return kx_, ky_, K2


def grid_U(qk, K_d2, K2, kx_, ky_, shear_strength=0.0):
    """grid_U.m:1-18 (6th argument defaults to 0: the 5-arg call sites at
    qgsw_raytrace.m:63,141-142 predate it).  Returns dict of 6 grid fields."""
    qk = np.asarray(qk, dtype=np.complex128)
    if qk.ndim == 3:
        K2b, kxb, kyb = K2[:, :, None], kx_[:, :, None], ky_[:, :, None]
    else:
        K2b, kxb, kyb = K2, kx_, ky_
    psik = -qk / (K_d2 + K2b)
    vk = 1j * kxb * psik
    uk = -1j * kyb * psik
    ukx = 1j * kxb * uk
    uky = 1j * kyb * uk
    vkx = 1j * kxb * vk
    vky = 1j * kyb * vk
    return {
        "u": apply_3d(uk, k2g) + shear_strength,
        "v": apply_3d(vk, k2g),
        "ux": apply_3d(ukx, k2g),
        "uy": apply_3d(uky, k2g),
        "vx": apply_3d(vkx, k2g),
        "vy": apply_3d(vky, k2g),
    }


def spectral_scheme_fields(L, nx, psi_field):
    """SpectralScheme.m:6-36 constructor: psi grid -> 7 grid fields.

    Integer wavenumbers regardless of L (SpectralScheme.m:12-13)."""
    kmax = nx // 2 - 1
    kx_, ky_ = np.meshgrid(np.arange(-kmax, kmax + 1, dtype=np.float64),
                           np.arange(0, kmax + 1, dtype=np.float64), indexing="ij")
    psik = g2k(psi_field)
    ugk = -1j * ky_ * psik
    vgk = 1j * kx_ * psik
    ugxk = 1j * kx_ * ugk
    ugyk = 1j * ky_ * ugk
    vgxk = 1j * kx_ * vgk
    vgyk = 1j * ky_ * vgk
    return {
        "psi": k2g(psik),
        "u": k2g(ugk),
        "v": k2g(vgk),
        "ux": k2g(ugxk),
        "uy": k2g(ugyk),
        "vx": k2g(vgxk),
        "vy": k2g(vgyk),
    }


FIELD_ORDER = ("u", "v", "ux", "uy", "vx", "vy")


# ----------------------------------------------------------------------------
# L2 — periodic 6x6 Lagrange interpolation (interpolate.m:1-50)
# ----------------------------------------------------------------------------
def lagrange_weights(a, bump):
    """interpolate.m:33-41: w(i) = prod_{j!=i} (a - j + bump)/(j - i), i,j in -2..3.

    Evaluated exactly in the reference order (j inner, running product,
    multiply-then-divide)."""
    a = np.asarray(a, dtype=np.float64)
    w = [np.ones_like(a) for _ in range(2 * (IORD + 1))]
    for i in range(-IORD, IORD + 2):
        for j in range(-IORD, IORD + 2):
            if i != j:
                w[i + IORD] = w[i + IORD] * (a - float(j) + bump) / float(j - i)
    return w


def _cell_and_frac(x, dx, period):
    """interpolate.m:21-31: xl = mod(x/dx, n); i0 = 1+floor(xl); a = 1+xl-i0.

    Returns 0-based cell index (i0-1, may equal `period` after round-up of
    mod) and the fractional offset a."""
    xl = matlab_mod(np.asarray(x, dtype=np.float64) / dx, float(period))
    fl = np.floor(xl)
    i0 = 1.0 + fl
    a = (1.0 + xl) - i0
    return fl.astype(np.int64), a


def interpolate(x, y, F, dx, dy, bump=BUMP_QG):
    """interpolate.m:1-50 vectorised over packets (per-packet arithmetic is
    bit-identical to the scalar loop: same ops, same order).

    F: nx x ny grid (first index = x).  A 3-D nx x nx x nz F reproduces the
    2-layer call (CS3): [nx,ny]=size(F) gives ny = nx*nz for the y-mod and
    2-subscript F(ig,jg) with jg<=nx reads layer 1."""
    F = np.asarray(F, dtype=np.float64)
    nx = F.shape[0]
    ny = int(np.prod(F.shape[1:]))
    F2 = F if F.ndim == 2 else F[:, :, 0]
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    shape = x.shape
    x = x.ravel()
    y = y.ravel()
    ic, ax = _cell_and_frac(x, dx, nx)
    jc, ay = _cell_and_frac(y, dy, ny)
    wx = lagrange_weights(ax, bump)
    wy = lagrange_weights(ay, bump)
    FI = np.zeros_like(x)
    for i in range(-IORD, IORD + 2):
        ig = np.mod(ic + i, nx)  # ig = 1 + mod(i0 + i - 1, nx)
        for j in range(-IORD, IORD + 2):
            jg = np.mod(jc + j, nx)  # jg = 1 + mod(j0 + j - 1, nx)  (nx, not ny: :46)
            FI = FI + wx[i + IORD] * wy[j + IORD] * F2[ig, jg]
    return FI.reshape(shape)


def interpolate_fields(x, y, fields, dx, bump, nyF=None):
    """Interpolate the 6 fields (FIELD_ORDER) at the points: 6 x N array.

    Same arithmetic as 6 calls of `interpolate` (the Lagrange weights and the
    2-D weight products are identical across calls)."""
    return np.stack([interpolate(x, y, _as_F(fields[name], nyF), dx, dx, bump)
                     for name in FIELD_ORDER])


def _as_F(f, nyF):
    f = np.asarray(f, dtype=np.float64)
    if nyF is None or f.ndim == 3:
        return f
    nz = nyF // f.shape[0]
    if nz == 1:
        return f
    # present as a 3-D array so interpolate() uses ny = nz*nx in the y-mod
    out = np.zeros(f.shape + (nz,))
    out[:, :, 0] = f
    return out


def interpolate_U(flow1, flow2, alpha, x, h, bump=BUMP_QG, nyF=None):
    """interpolate_U.m:1-24 — 12 interpolations and the linear time blend.

    x: N x 2.  Returns U (N x 2) and dict u_x,u_y,v_x,v_y (N,)."""
    xx = x[:, 0]
    yy = x[:, 1]
    I1 = {n: interpolate(xx, yy, _as_F(flow1[n], nyF), h, h, bump) for n in FIELD_ORDER}
    I2 = {n: interpolate(xx, yy, _as_F(flow2[n], nyF), h, h, bump) for n in FIELD_ORDER}
    U1 = np.stack([I1["u"], I1["v"]], axis=1)
    U2 = np.stack([I2["u"], I2["v"]], axis=1)
    U = (1 - alpha) * U1 + alpha * U2
    nab = {
        "u_x": (1 - alpha) * I1["ux"] + alpha * I2["ux"],
        "u_y": (1 - alpha) * I1["uy"] + alpha * I2["uy"],
        "v_x": (1 - alpha) * I1["vx"] + alpha * I2["vx"],
        "v_y": (1 - alpha) * I1["vy"] + alpha * I2["vy"],
    }
    return U, nab


# ----------------------------------------------------------------------------
# L2 boundary API — RaytracingScheme.m / SpectralScheme.m
# ----------------------------------------------------------------------------
class SpectralSchemeOracle:
    """SpectralScheme(L, nx, psi_field) (SpectralScheme.m:1-70) + the concrete
    RaytracingScheme methods (RaytracingScheme.m:9-26).

    `interpolate` resolves to ray_trace_sw/interpolate.m after the
    constructor's addpath (CS2), hence bump = 1e-13."""

    def __init__(self, L, nx, psi_field, bump=BUMP_SW):
        self.L = L
        self.nx = nx
        self.bump = bump
        fl = spectral_scheme_fields(L, nx, psi_field)
        self.psi_field = fl.pop("psi")
        self.fields = fl  # u, v, ux, uy, vx, vy

    @property
    def dx(self):
        return self.L / self.psi_field.shape[0]  # SpectralScheme.m:46

    def streamfunction(self, x, y, t=0.0):
        return interpolate(x, y, self.psi_field, self.dx, self.dx, self.bump)

    def U(self, x, t=0.0):
        """x: M x 2 x P (or N x 2) -> same shape (SpectralScheme.m:45-54)."""
        x = np.asarray(x, dtype=np.float64)
        xx = x[:, 0, ...]
        yy = x[:, 1, ...]
        u = np.zeros_like(x)
        u[:, 0, ...] = interpolate(xx, yy, self.fields["u"], self.dx, self.dx, self.bump)
        u[:, 1, ...] = interpolate(xx, yy, self.fields["v"], self.dx, self.dx, self.bump)
        return u

    def grad_U(self, x, t=0.0):
        """SpectralScheme.m:56-68 — struct of column vectors (numel(x)/2)."""
        x = np.asarray(x, dtype=np.float64)
        xx = np.ravel(x[:, 0, ...], order="F")
        yy = np.ravel(x[:, 1, ...], order="F")
        d = self.dx
        return {
            "u_x": interpolate(xx, yy, self.fields["ux"], d, d, self.bump),
            "u_y": interpolate(xx, yy, self.fields["uy"], d, d, self.bump),
            "v_x": interpolate(xx, yy, self.fields["vx"], d, d, self.bump),
            "v_y": interpolate(xx, yy, self.fields["vy"], d, d, self.bump),
        }

    def grad_U_times_k(self, x, k, t=0.0):
        """RaytracingScheme.m:9-16."""
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


# ----------------------------------------------------------------------------
# L3 — ode_symplectic.m (Strang / leapfrog)
# ----------------------------------------------------------------------------
def _omega(k1, k2, f, gH):
    """ode_symplectic.m:10 — sqrt(f^2 + gH*dot(k,k,2))."""
    return np.sqrt(f * f + gH * (k1 * k1 + k2 * k2))


def ode_symplectic(x0, k0, dt, T, f, gH, scheme):
    """ode_symplectic.m:1-31 verbatim semantics.  x0, k0: 1 x 2 x P.

    Returns x, k: Nsteps x 2 x P and t: (Nsteps,)."""
    Nsteps = int(math.floor(T / dt))
    x0 = np.array(x0, dtype=np.float64)
    k0 = np.array(k0, dtype=np.float64)
    P = x0.shape[2]
    x = np.zeros((Nsteps, 2, P))
    k = np.zeros((Nsteps, 2, P))
    t = np.zeros(Nsteps)
    x[0] = x0[0]
    k[0] = k0[0]

    def group_velocity(kk):
        w = _omega(kk[:, 0:1, :], kk[:, 1:2, :], f, gH)
        return gH * kk / w

    def phi1(xa, ka, h):
        return xa + h * group_velocity(ka), ka

    def phi2(xa, ka, h):
        return xa + h * scheme.U(xa), ka - h * scheme.grad_U_times_k(xa, ka, 0)

    for i in range(1, Nsteps):
        x1, k1 = phi1(x0, k0, dt / 2)
        x2, k2 = phi2(x1, k1, dt)
        x0, k0 = phi1(x2, k2, dt / 2)
        x[i] = x0[0]
        k[i] = k0[0]
        t[i] = i * dt
    return x, k, t


@dataclass
class GridField:
    """Six gridded fields (u, v, u_x, u_y, v_x, v_y) of one snapshot.

    nyF is the y-period used by interpolate's mod (nx for 1 layer, nz*nx for
    the 2-layer call of qg2layersw_raytrace.m:187-188)."""
    fields: dict
    dx: float
    nyF: int | None = None


def leapfrog(x, k, dt, nsteps, f, gH, snap0: GridField, snap1: GridField | None = None,
             alpha0=0.0, dalpha=0.0, bump=BUMP_SW, save_every=0):
    """Vectorised `ode_symplectic` inner loop (ode_symplectic.m:23-37) on
    N x 2 state, generalised to a two-snapshot time blend: the kick of step s
    evaluates U, grad U with interpolate_U's blend (interpolate_U.m:19-23) at
    alpha = alpha0 + s*dalpha.  With snap1=None this is exactly the steady
    SpectralScheme path (scheme time 0).

    Returns (x, k, hist_x, hist_k): hist frames are N x 2 arrays after every
    `save_every` steps (packet_x.bin frame layout, write_field.m:38)."""
    x = np.array(x, dtype=np.float64)
    k = np.array(k, dtype=np.float64)
    hx, hk = [], []
    half = dt / 2
    for s in range(nsteps):
        # phi1(x0, k0, dt/2)
        w = _omega(k[:, 0], k[:, 1], f, gH)
        x1 = np.stack([x[:, 0] + half * (gH * k[:, 0] / w),
                       x[:, 1] + half * (gH * k[:, 1] / w)], axis=1)
        # phi2(x1, k1, dt): U and grad U at x1
        if snap1 is None:
            I = interpolate_fields(x1[:, 0], x1[:, 1], snap0.fields, snap0.dx, bump, snap0.nyF)
            u, v, ux, uy, vx, vy = I
        else:
            alpha = alpha0 + s * dalpha
            U, nab = interpolate_U(snap0.fields, snap1.fields, alpha, x1, snap0.dx, bump, snap0.nyF)
            u, v = U[:, 0], U[:, 1]
            ux, uy, vx, vy = nab["u_x"], nab["u_y"], nab["v_x"], nab["v_y"]
        k1, l1 = k[:, 0], k[:, 1]
        x2 = np.stack([x1[:, 0] + dt * u, x1[:, 1] + dt * v], axis=1)
        k2 = np.stack([k1 - dt * (ux * k1 + vx * l1), l1 - dt * (uy * k1 + vy * l1)], axis=1)
        # phi1(x2, k2, dt/2)
        w = _omega(k2[:, 0], k2[:, 1], f, gH)
        x = np.stack([x2[:, 0] + half * (gH * k2[:, 0] / w),
                      x2[:, 1] + half * (gH * k2[:, 1] / w)], axis=1)
        k = k2
        if save_every and (s + 1) % save_every == 0:
            hx.append(x.copy())
            hk.append(k.copy())
    return x, k, hx, hk


# ----------------------------------------------------------------------------
# Exact Fourier-mode kick (scratch/fourier_interpolate_test.m:92-136) — KAT source
# ----------------------------------------------------------------------------
def fourier_velocity(x, y, amp, phase, n):
    """fourier_interpolate_test.m:125-136: U for psi = sum A cos(Kx+Ly+phi)."""
    u = np.zeros_like(x, dtype=np.float64)
    v = np.zeros_like(y, dtype=np.float64)
    for K in range(-n, n + 1):
        for Lw in range(-n, n + 1):
            a = amp[K + n, Lw + n]
            s = np.sin(K * x + Lw * y + phase[K + n, Lw + n])
            u = u + -Lw * a * -s
            v = v + K * a * -s
    return u, v


def fourier_streamfunction(X, Y, amp, phase, n):
    """fourier_interpolate_test.m:116-123."""
    psi = np.zeros_like(X, dtype=np.float64)
    for K in range(-n, n + 1):
        for Lw in range(-n, n + 1):
            psi = psi + amp[K + n, Lw + n] * np.cos(K * X + Lw * Y + phase[K + n, Lw + n])
    return psi


def fourier_grad(x, y, amp, phase, n):
    """Closed-form grad U of the same field (u = -psi_y, v = psi_x)."""
    ux = np.zeros_like(x); uy = np.zeros_like(x); vx = np.zeros_like(x); vy = np.zeros_like(x)
    for K in range(-n, n + 1):
        for Lw in range(-n, n + 1):
            a = amp[K + n, Lw + n]
            c = np.cos(K * x + Lw * y + phase[K + n, Lw + n])
            # psi = a cos(th): psi_x = -aK sin, psi_y = -aL sin
            # u = -psi_y = aL sin -> u_x = aLK cos, u_y = aL^2 cos
            # v = psi_x = -aK sin -> v_x = -aK^2 cos, v_y = -aKL cos
            ux = ux + a * Lw * K * c
            uy = uy + a * Lw * Lw * c
            vx = vx - a * K * K * c
            vy = vy - a * K * Lw * c
    return ux, uy, vx, vy


def fourier_phi2(x0, k0, dt, amp, phase, n):
    """fourier_interpolate_test.m:92-114 exact kick (x0,k0: N x 2)."""
    xx, yy = x0[:, 0], x0[:, 1]
    kk, ll = k0[:, 0], k0[:, 1]
    ux_ = np.zeros_like(xx); uy_ = np.zeros_like(xx); uk_ = np.zeros_like(xx); ul_ = np.zeros_like(xx)
    for K in range(-n, n + 1):
        for Lw in range(-n, n + 1):
            c = K * xx + Lw * yy
            a = Lw * kk - K * ll
            A = amp[K + n, Lw + n]
            ph = phase[K + n, Lw + n]
            ux_ = ux_ - dt * Lw * A * -np.sin(c + ph)
            uy_ = uy_ + dt * K * A * -np.sin(c + ph)
            uk_ = uk_ + dt * K * A * -np.cos(c + ph) * a
            ul_ = ul_ + dt * Lw * A * -np.cos(c + ph) * a
    return (np.stack([xx + ux_, yy + uy_], axis=1), np.stack([kk + uk_, ll + ul_], axis=1))


# ----------------------------------------------------------------------------
# I/O — write_field.m / read_field.m (raw native-endian fp64, appended frames)
# ----------------------------------------------------------------------------
def write_field(field, fname, frame=1):
    """write_field.m:22-49: append column-major fp64 frame; complex = re then im."""
    field = np.asarray(field)
    with open(str(fname) + ".bin", "ab") as fh:
        if np.iscomplexobj(field):
            fh.write(np.asfortranarray(field.real, dtype=np.float64).tobytes(order="F"))
            fh.write(np.asfortranarray(field.imag, dtype=np.float64).tobytes(order="F"))
        else:
            fh.write(np.asarray(field, dtype=np.float64).tobytes(order="F"))


def read_field(fname, nx=1, ny=1, nz=1, frames=None):
    """read_field.m:58-101 for real fields: returns nx x ny (x nz) x frames."""
    data = np.fromfile(str(fname) + ".bin", dtype=np.float64)
    if nx == 1:
        return data[None, :]
    per = nx * ny * nz
    nfr = data.size // per
    frames = list(range(1, nfr + 1)) if frames is None else list(frames)
    out = np.stack([data[(fr - 1) * per: fr * per].reshape((nx, ny, nz), order="F") for fr in frames],
                   axis=-1)
    return np.squeeze(out)


# ----------------------------------------------------------------------------
# Synthetic inputs (qgsw_raytrace.m:191-214, :54-60) with a numpy RNG
# ----------------------------------------------------------------------------
def initial_q(nx, L, a_g, K_d2, k_min, k_max, rng):
    """initial_q (qgsw_raytrace.m:191-214; k in (5,8]; 2-layer: (10,30],
    qg2layersw_raytrace.m:258-281).  Grid X,Y = meshgrid(linspace(-L/2,L/2,nx))
    as in the reference (note: linspace includes both ends, not periodic)."""
    xs = np.linspace(-L / 2, L / 2, nx)
    X, Y = np.meshgrid(xs, xs)  # qgsw_raytrace.m:15-16 (meshgrid)
    q = 0 * X
    U = 0 * X
    V = 0 * X
    phase = 2 * np.pi * rng.random((2 * k_max + 1, 2 * k_max + 1))
    for k in range(-k_max, k_max + 1):
        for l in range(-k_max, k_max + 1):
            if k_min**2 < k**2 + l**2 <= k_max**2:
                wave_phase = k * X + l * Y + phase[k + k_max, l + k_max]
                U = U - l * np.sin(wave_phase)
                V = V + k * np.sin(wave_phase)
                q = q - (K_d2 + k**2 + l**2) * np.cos(wave_phase)
    speed2 = U**2 + V**2
    return a_g / np.sqrt(speed2.max()) * q


def initial_packets(N, L, near_inertial_factor, f, Cg, rng):
    """qgsw_raytrace.m:54-60: k on a ring, x uniform in [-L/2, L/2)^2."""
    wf = math.sqrt((near_inertial_factor**2 - 1) * f**2 / Cg**2)
    i = np.arange(1, N + 1, dtype=np.float64)
    k = np.stack([wf * np.cos(2 * np.pi * i / N), wf * np.sin(2 * np.pi * i / N)], axis=1)
    x = L * rng.random((N, 2)) - L / 2
    return x, k


def here():
    return os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------
# ray_trace_sw/step_packet_xka.m + cg_sw.m (wave action, RSW background)
# ----------------------------------------------------------------------------
def cg_sw(k, l, C0, f, U, H=None):
    """cg_sw.m:1-32 on full fields (k, l scalars; U dict u, v; H field).

    Returns C (dict x, y), omega, omega_abs, divC, gradomega (dict x, y)."""
    if H is not None:
        gH = C0 ** 2 * np.asarray(H, dtype=np.float64)  # cg_sw.m:15-16
    else:
        gH = C0 ** 2
    K2 = k ** 2 + l ** 2
    omega = np.sqrt(f ** 2 + gH * K2)  # cg_sw.m:22
    omega_abs = np.abs(omega)
    C = {"x": gH * k / omega, "y": gH * l / omega}  # cg_sw.m:25-26
    divC = gradomega = None
    if U is not None:  # cg_sw.m:28-32
        divC = (k * f * U["v"] - l * f * U["u"] - C["x"] ** 2 - C["y"] ** 2) / omega
        gradomega = {"x": f * K2 * U["v"] / (2 * omega), "y": -f * K2 * U["u"] / (2 * omega)}
    return C, omega, omega_abs, divC, gradomega


def step_packet_xka(P, U, GradU, H, C0, f, dx, dy, dt):
    """step_packet_xka.m:1-91 for one packet P = dict(x, y, k, l, a) (floats).

    Literal restatement: cg_sw on the full fields with the packet's k, l, RK4 of
    x through interpolate(U.u + C.x) (k frozen), then 7 interpolations at the new
    position and RK4 of k, l and the action a with frozen coefficients.
    `interpolate` is ray_trace_sw/interpolate.m (bump 1e-13)."""
    b = BUMP_SW
    C, _, _, divC, gw = cg_sw(P["k"], P["l"], C0, f, U, H)
    Fu = U["u"] + C["x"]
    Fv = U["v"] + C["y"]

    def I(x, y, F):
        return float(interpolate(np.array([x]), np.array([y]), F, dx, dy, b)[0])

    x, y = P["x"], P["y"]
    x1 = dt * I(x, y, Fu)
    y1 = dt * I(x, y, Fv)
    x2 = dt * I(x + x1 / 2, y + y1 / 2, Fu)
    y2 = dt * I(x + x1 / 2, y + y1 / 2, Fv)
    x3 = dt * I(x + x2 / 2, y + y2 / 2, Fu)
    y3 = dt * I(x + x2 / 2, y + y2 / 2, Fv)
    x4 = dt * I(x + x3, y + y3, Fu)
    y4 = dt * I(x + x3, y + y3, Fv)
    out = {}
    out["x"] = x + (x1 + 2 * x2 + 2 * x3 + x4) / 6
    out["y"] = y + (y1 + 2 * y2 + 2 * y3 + y4) / 6
    X, Y = out["x"], out["y"]
    u_xi = I(X, Y, GradU["u_x"])
    u_yi = I(X, Y, GradU["u_y"])
    v_xi = I(X, Y, GradU["v_x"])
    v_yi = I(X, Y, GradU["v_y"])
    omega_xi = I(X, Y, gw["x"])
    omega_yi = I(X, Y, gw["y"])
    divCi = I(X, Y, divC)
    k, l = P["k"], P["l"]
    k1 = dt * (-u_xi * k - v_xi * l - omega_xi)
    l1 = dt * (-u_yi * k - v_yi * l - omega_yi)
    k2 = dt * (-u_xi * (k + k1 / 2) - v_xi * (l + l1 / 2) - omega_xi)
    l2 = dt * (-u_yi * (k + k1 / 2) - v_yi * (l + l1 / 2) - omega_yi)
    k3 = dt * (-u_xi * (k + k2 / 2) - v_xi * (l + l2 / 2) - omega_xi)
    l3 = dt * (-u_yi * (k + k2 / 2) - v_yi * (l + l2 / 2) - omega_yi)
    k4 = dt * (-u_xi * (k + k3) - v_xi * (l + l3) - omega_xi)
    l4 = dt * (-u_yi * (k + k3) - v_yi * (l + l3) - omega_yi)
    out["k"] = k + (k1 + 2 * k2 + 2 * k3 + k4) / 6
    out["l"] = l + (l1 + 2 * l2 + 2 * l3 + l4) / 6
    a = P["a"]
    a1 = dt * (-a * divCi)
    a2 = dt * (-(a + a1 / 2) * divCi)
    a3 = dt * (-(a + a2 / 2) * divCi)
    a4 = dt * (-(a + a3) * divCi)
    out["a"] = a + (a1 + 2 * a2 + 2 * a3 + a4) / 6
    return out


def rsw_background(S, f, Cg, L=2 * math.pi):
    """ray_trace_sw/raytrace_sw.m:16-52: geostrophic part of an RSW state.

    S: nx x nx x 3 grid state [u v eta] (raytrace_sw.m:12).  The script's
    integer wavenumbers are those of L = 2*pi (:84); another period scales
    them by 2*pi/L (exactly 1.0 at 2*pi, so the script's values are
    unchanged).  Returns dict(U={u, v}, GradU={u_x, u_y, v_x, v_y},
    H = 1 + eta_g, etag), the inputs of step_packet_xka."""
    S = np.asarray(S, dtype=np.float64)
    nx = S.shape[0]
    kx_, ky_, _ = wavenumber_grids(nx)  # :16-18
    ks = (2 * math.pi) / L
    kx_, ky_ = kx_ * ks, ky_ * ks
    K2_ = kx_ ** 2 + ky_ ** 2
    gH0 = Cg ** 2  # :22
    sig2_ = f ** 2 + gH0 * K2_  # :25
    uk = g2k(S[:, :, 0])  # :26-28
    vk = g2k(S[:, :, 1])
    etak = g2k(S[:, :, 2])
    zetak = 1j * (kx_ * vk - ky_ * uk)  # :29
    etagk = (f * etak - zetak) * f / sig2_  # :30
    ugk = (-1j * ky_) * (gH0 / f * etagk)  # :34
    vgk = (1j * kx_) * (gH0 / f * etagk)  # :35
    ugxk = (1j * kx_) * ugk  # :38-41
    ugyk = (1j * ky_) * ugk
    vgxk = (1j * kx_) * vgk
    vgyk = (1j * ky_) * vgk
    etag = k2g(etagk)  # :44-52
    return dict(U={"u": k2g(ugk), "v": k2g(vgk)},
                GradU={"u_x": k2g(ugxk), "u_y": k2g(ugyk), "v_x": k2g(vgxk), "v_y": k2g(vgyk)},
                H=1 + etag, etag=etag)


def childress_soward(nx, U0=0.1, km=4.0, a=0.25, L=2 * math.pi):
    """ray_trace_sw/raytrace.m:30-37 analytic cellular flow on the grid
    x = (0:nx-1)*dx (raytrace.m:26-28): returns U, GradU dicts."""
    x = np.arange(nx) * (L / nx)
    X, Y = np.meshgrid(x, x, indexing="ij")
    s, c = np.sin, np.cos
    U = {"u": -U0 * (s(km * X) * c(km * Y) - a * c(km * X) * s(km * Y)),
         "v": U0 * (c(km * X) * s(km * Y) - a * s(km * X) * c(km * Y))}
    G = {"u_x": -km * U0 * (c(km * X) * c(km * Y) + a * s(km * X) * s(km * Y)),
         "u_y": km * U0 * (s(km * X) * s(km * Y) + a * c(km * X) * c(km * Y)),
         "v_x": -km * U0 * (s(km * X) * s(km * Y) + a * c(km * X) * c(km * Y)),
         "v_y": km * U0 * (c(km * X) * c(km * Y) + a * s(km * X) * s(km * Y))}
    return U, G


# ----------------------------------------------------------------------------
# Exact spectral evaluator (scratch/fourier_interpolate_test.m:92-136 generalised)
# ----------------------------------------------------------------------------
def spectral_direct(C, kx0, ky0, s, x, y):
    """psi = sum Re(C[i,j] e^{i(kx_i x + ky_j y)}): returns 6 x N flow
    (u, v, u_x, u_y, v_x, v_y) with u = -psi_y, v = psi_x (direct sincos sum)."""
    C = np.asarray(C, dtype=np.complex128)
    x = np.asarray(x, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    nkx, nky = C.shape
    kx = (kx0 + np.arange(nkx)) * s
    ky = (ky0 + np.arange(nky)) * s
    px = np.zeros_like(x); py = np.zeros_like(x)
    pxx = np.zeros_like(x); pxy = np.zeros_like(x); pyy = np.zeros_like(x)
    Ex = np.exp(1j * np.outer(x, kx))  # N x nkx
    for j in range(nky):
        z = (Ex * np.exp(1j * ky[j] * y)[:, None]) * C[None, :, j]  # N x nkx
        px += -(z.imag * kx).sum(axis=1)
        py += -ky[j] * z.imag.sum(axis=1)
        pxx += -(z.real * kx * kx).sum(axis=1)
        pxy += -ky[j] * (z.real * kx).sum(axis=1)
        pyy += -ky[j] ** 2 * z.real.sum(axis=1)
    return np.stack([-py, px, -pxy, -pyy, pxx, pxy])


def modes_from_halfplane(fk, k_scale=1.0):
    """g2k half plane -> dense coefficient grid of the spectral evaluator
    (k2g's point formula): C = 2 fk, ky=0/kx<0 zeroed, DC real."""
    fk = np.asarray(fk, dtype=np.complex128)
    kmax = fk.shape[1] - 1
    C = 2 * fk
    C[:kmax, 0] = 0
    C[kmax, 0] = fk[kmax, 0].real
    return C, -kmax, 0, k_scale


def modes_from_amp_phase(amp, phase, n):
    """fourier_interpolate_test.m:116-123 field: C = amp .* exp(1i*phase), K, L in -n..n."""
    return np.asarray(amp) * np.exp(1j * np.asarray(phase)), -n, -n, 1.0


# ----------------------------------------------------------------------------
# QG PDE steppers — the step BEFORE the packet path
#   1-layer: qg_flow_ray_trace/qgsw_raytrace.m:111-137 (AB3 + filter),
#            update :270-286, inertial_ring :216-220, filter :222-230
#   2-layer: qg_flow_ray_trace/qg2layersw_raytrace.m:129-181 (exponential
#            AB3, adaptive CFL), update :309-323, mmult3 :333-338,
#            diag_exp :340-343
# ----------------------------------------------------------------------------
def inertial_ring(force_strength, K2, f, Cg):
    """qgsw_raytrace.m:216-220."""
    omega = np.sqrt(f**2 + Cg**2 * K2)
    forces = np.zeros(K2.shape)
    forces[(0.9 * f < omega) & (omega < 1.1 * f)] = force_strength
    return forces


def qg_filter(kx_, ky_, dx):
    """qgsw_raytrace.m:222-230 (exponential cutoff filter above kc = 0.75 pi)."""
    Ef = np.ones(kx_.shape)
    kstar = np.sqrt((kx_ * dx) ** 2 + (ky_ * dx) ** 2)
    kc = 0.75 * np.pi
    const = np.log(1e-15) / (0.25 * np.pi) ** 4
    result = np.exp(const * (kstar - kc) ** 4)
    sel = kstar >= kc
    Ef[sel] = result[sel]
    return Ef


def _jacobian_term(psik, qk, kx_, ky_):
    """J = psix.*qy - psiy.*qx on the grid (update at qgsw_raytrace.m:271-282 /
    qg2layersw_raytrace.m:311-321), one layer."""
    psix = k2g(1j * kx_ * psik)
    psiy = k2g(1j * ky_ * psik)
    qx = k2g(1j * kx_ * qk)
    qy = k2g(1j * ky_ * qk)
    return psix * qy - psiy * qx


def qg1_update(qk, K2, K_d2, beta, r_drag, surface_forces, kx_, ky_):
    """qgsw_raytrace.m:270-286 (including its r_drag*K2 and surface_forces terms
    exactly as written)."""
    psik = -qk / (K_d2 + K2)
    psikx = 1j * kx_ * psik
    J = _jacobian_term(psik, qk, kx_, ky_)
    return g2k(J) - beta * psikx + r_drag * K2 + surface_forces


class QG1Oracle:
    """qgsw_raytrace.m:111-137: AB3 (Euler, AB2 start) then the filter."""

    def __init__(self, qk, nx, K_d2, beta=0.0, r_drag=0.1, force_strength=0.1, f=3.0, Cg=1.0,
                 use_filter=True):
        self.kx, self.ky, self.K2 = wavenumber_grids(nx)
        self.nx = nx
        self.dx = 2 * np.pi / nx
        self.qk = np.array(qk, dtype=np.complex128)
        self.K_d2, self.beta, self.r_drag = K_d2, beta, r_drag
        self.forces = inertial_ring(force_strength, self.K2, f, Cg)
        self.Ef = qg_filter(self.kx, self.ky, self.dx) if use_filter else np.ones(self.K2.shape)
        self.Qm = [np.zeros_like(self.qk), np.zeros_like(self.qk)]
        self.step_no = 0
        self.t = 0.0

    def step(self, dt):
        self.step_no += 1
        Qn = qg1_update(self.qk, self.K2, self.K_d2, self.beta, self.r_drag, self.forces, self.kx, self.ky)
        if self.step_no == 1:
            dq = dt * Qn
        elif self.step_no == 2:
            dq = dt / 2 * (3 * Qn - self.Qm[0])
        else:
            dq = dt / 12 * (23 * Qn - 16 * self.Qm[0] + 5 * self.Qm[1])
        self.t = self.t + dt
        self.Qm[1] = self.Qm[0]
        self.Qm[0] = Qn
        self.qk = self.qk + dq
        self.qk = self.Ef * self.qk


def mmult3(A, x):
    """qg2layersw_raytrace.m:333-338: y(:,:,i) = A(i,1).*x(:,:,1) + A(i,2).*x(:,:,2).
    A: (2, 2, nkx, nky), x: (nkx, nky, 2)."""
    y = np.zeros(x.shape, dtype=np.complex128)
    for i in range(2):
        y[:, :, i] = A[i, 0] * x[:, :, 0] + A[i, 1] * x[:, :, 1]
    return y


def qg2_operators(nx, L, K_d2, beta, shear_strength, nu, alpha, r):
    """qg2layersw_raytrace.m:129-147: B (PV inversion), factor_L and its
    eigen-decomposition (pageeig / pageinv)."""
    kx_, ky_, K2 = wavenumber_grids(nx, L, scale=True)
    F = K_d2 / 2
    B = np.zeros((2, 2) + K2.shape)
    B[0, 0] = -F - K2
    B[0, 1] = -F
    B[1, 0] = -F
    B[1, 1] = -F - K2
    detB = K2 * (K2 + 2 * F)
    detB[K2 == 0] = np.inf
    B = B / detB
    diffusion_factor = (nu * K2**alpha + r) * K2 - 1j * kx_ * beta
    diffusion_terms = B * diffusion_factor
    shear_factor = 1j * kx_ * shear_strength
    # pagemtimes([-1,0;0,1], eye(2) + 2*F*B)
    IB = np.zeros((2, 2) + K2.shape)
    IB[0, 0] = 1 + 2 * F * B[0, 0]
    IB[0, 1] = 2 * F * B[0, 1]
    IB[1, 0] = 2 * F * B[1, 0]
    IB[1, 1] = 1 + 2 * F * B[1, 1]
    S = np.array([[-1.0, 0.0], [0.0, 1.0]])
    MF = np.einsum("ij,jk...->ik...", S, IB)
    factor_L = shear_factor * MF + diffusion_terms
    Lp = np.moveaxis(factor_L, (0, 1), (-2, -1))  # pages last
    LD, LV = np.linalg.eig(Lp)
    LV1 = np.linalg.inv(LV)
    return dict(kx=kx_, ky=ky_, K2=K2, B=B, factor_L=factor_L, LD=LD, LV=LV, LV1=LV1)


def qg2_expL(ops, dt):
    """LV * diag(exp(dt*LD)) * LV^-1 per wavenumber (qg2layersw_raytrace.m:148,
    diag_exp :340-343), as (2, 2, nkx, nky)."""
    E = ops["LV"] * np.exp(dt * ops["LD"])[..., None, :]
    M = E @ ops["LV1"]
    return np.moveaxis(M, (-2, -1), (0, 1))


def qg2_update(qk, B, kx_, ky_):
    """qg2layersw_raytrace.m:309-323."""
    psik = mmult3(B, qk)
    dq = np.zeros_like(qk)
    for i in range(2):
        dq[:, :, i] = g2k(_jacobian_term(psik[:, :, i], qk[:, :, i], kx_, ky_))
    return dq


class QG2Oracle:
    """qg2layersw_raytrace.m:129-181: exponential AB3 with the adaptive CFL rule
    of :156-165 (grid_U of both layers, u += shear_strength)."""

    def __init__(self, qk, nx, L, K_d2, beta=0.0, shear_strength=0.5, nu=None, alpha=4, r=0.4,
                 nutune=0.1, cfl_fraction=0.25):
        self.nx, self.L = nx, L
        self.dx = L / nx
        self.K_d2, self.shear = K_d2, shear_strength
        self.nu = nutune * self.dx ** (2 * alpha) if nu is None else nu
        self.ops = qg2_operators(nx, L, K_d2, beta, shear_strength, self.nu, alpha, r)
        self.qk = np.array(qk, dtype=np.complex128)
        self.cfl = cfl_fraction
        self.U0 = self.max_speed()
        self.dt = cfl_fraction * self.dx / self.U0  # qg2layersw_raytrace.m:78
        self.exps(self.dt)
        self.Qm = [np.zeros_like(self.qk), np.zeros_like(self.qk)]
        self.step_no = 0
        self.t = 0.0

    def exps(self, dt):
        self.expLdt = qg2_expL(self.ops, dt)
        self.expL2dt = qg2_expL(self.ops, 2 * dt)

    def max_speed(self):
        o = self.ops
        flow = grid_U(self.qk, self.K_d2, o["K2"], o["kx"], o["ky"], self.shear)
        return float(np.sqrt((flow["u"] ** 2 + flow["v"] ** 2).max()))

    def cfl_check(self):
        """qg2layersw_raytrace.m:156-165; returns True when dt changed."""
        self.U0 = self.max_speed()
        cond = self.cfl * self.dx / self.U0
        if cond < self.dt or self.dt < cond / 4:
            self.dt = self.cfl / 2 * self.dx / self.U0
            self.exps(self.dt)
            return True
        return False

    def step(self, dt=None):
        """One step; dt=None applies the adaptive CFL rule first (the driver),
        an explicit dt skips it (fixed-step use)."""
        if dt is None:
            self.cfl_check()
        elif dt != self.dt:
            self.dt = dt
            self.exps(dt)
        dt = self.dt
        self.step_no += 1
        Qn = qg2_update(self.qk, self.ops["B"], self.ops["kx"], self.ops["ky"])
        if self.step_no == 1:
            dq = dt * Qn
        elif self.step_no == 2:
            dq = dt / 2 * (3 * Qn - mmult3(self.expLdt, self.Qm[0]))
        else:
            dq = dt / 12 * (23 * Qn - 16 * mmult3(self.expLdt, self.Qm[0]) + 5 * mmult3(self.expL2dt, self.Qm[1]))
        self.t = self.t + dt
        self.Qm[1] = self.Qm[0]
        self.Qm[0] = Qn
        self.qk = mmult3(self.expLdt, self.qk + dq)


# ----------------------------------------------------------------------------
# ode23 — the production drivers' packet integrator (qgsw_raytrace.m:143-150,
# qg2layersw_raytrace.m:189-196).  MATLAB's ode23 is
# proprietary and not vendored: this restates its published algorithm
# (Bogacki-Shampine 3(2) pair, FSAL; Shampine & Reichelt, "The MATLAB ODE
# Suite", SIAM J. Sci. Comput. 18 (1997)) with R2020b's defaults RelTol 1e-3,
# AbsTol 1e-6, MaxStep 0.1*|tspan|, max-norm error control, the initial-step
# heuristic and the step-size update rules.  PARITY UNPINNED against MATLAB
# itself (no reference run or fixture exists); the GPU path is pinned to
# this restatement.
# ----------------------------------------------------------------------------
def raytracing_rhs(flow1, flow2, f, Cg, tmax, h, nyF=None, bump=BUMP_QG):
    """generate_raytracing_ode / odefun (qgsw_raytrace.m:258-268): y is the 4N
    column [x(:,1); x(:,2); k(:,1); k(:,2)] (ode_xk2y, :238-244)."""
    def odefun(t, y):
        n = y.size // 4
        x = np.stack([y[0:n], y[n:2 * n]], axis=1)
        k = np.stack([y[2 * n:3 * n], y[3 * n:4 * n]], axis=1)
        U, nab = interpolate_U(flow1, flow2, t / tmax, x, h, bump=bump, nyF=nyF)
        s = np.sqrt(f**2 + Cg**2 * (k[:, 0] * k[:, 0] + k[:, 1] * k[:, 1]))
        dxdt = U + (Cg * k) / s[:, None]
        dk1 = -(nab["u_x"] * k[:, 0] + nab["v_x"] * k[:, 1])
        dk2 = -(nab["u_y"] * k[:, 0] + nab["v_y"] * k[:, 1])
        return np.concatenate([dxdt[:, 0], dxdt[:, 1], dk1, dk2])
    return odefun


ODE23_A = (0.5, 0.75, 1.0)
ODE23_B3 = (2.0 / 9.0, 1.0 / 3.0, 4.0 / 9.0)
ODE23_E = (-5.0 / 72.0, 1.0 / 12.0, 1.0 / 9.0, -1.0 / 8.0)


def ode23(odefun, tspan, y0, rtol=1e-3, atol=1e-6, stats=None):
    """[t, y] = ode23(odefun, [t0 tfinal], y0) restricted to what the drivers
    use (scalar AbsTol, no events/mass/NonNegative, Refine irrelevant since
    only y(end) is consumed).  Returns (t_accepted, y_final)."""
    t0, tfinal = float(tspan[0]), float(tspan[1])
    tdir = math.copysign(1.0, tfinal - t0)
    pow_ = 1.0 / 3.0
    rtol = max(rtol, 100 * np.finfo(float).eps)
    threshold = atol / rtol
    htspan = abs(tfinal - t0)
    hmax = 0.1 * htspan
    t = t0
    y = np.array(y0, dtype=np.float64)
    f1 = odefun(t, y)
    # initial step (ode23.m: absh = min(hmax, htspan); rh = ...)
    absh = min(hmax, htspan)
    rh = np.max(np.abs(f1) / np.maximum(np.abs(y), threshold)) / (0.8 * rtol**pow_)
    if absh * rh > 1:
        absh = 1.0 / rh
    absh = max(absh, 16 * np.spacing(t))
    ts = [t]
    done = False
    nfailed = 0
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
            y2 = y + f1 * (h * 0.5)
            f2 = odefun(t + h * ODE23_A[0], y2)
            y3 = y + f2 * (h * 0.75)
            f3 = odefun(t + h * ODE23_A[1], y3)
            tnew = t + h * ODE23_A[2]
            if done:
                tnew = tfinal
            h = tnew - t
            ynew = y + (((f1 * (h * ODE23_B3[0])) + f2 * (h * ODE23_B3[1])) + f3 * (h * ODE23_B3[2]))
            f4 = odefun(tnew, ynew)
            fE = ((f1 * ODE23_E[0] + f2 * ODE23_E[1]) + f3 * ODE23_E[2]) + f4 * ODE23_E[3]
            err = absh * np.max(np.abs(fE) / np.maximum(np.maximum(np.abs(y), np.abs(ynew)), threshold))
            if err > rtol:
                nfailed += 1
                if absh <= hmin:
                    raise RuntimeError(f"ode23: step size {absh} below hmin at t={t}")
                if nofailed:
                    nofailed = False
                    absh = max(hmin, absh * max(0.5, 0.8 * (rtol / err) ** pow_))
                else:
                    absh = max(hmin, 0.5 * absh)
                h = tdir * absh
                done = False
            else:
                break
        t = tnew
        y = ynew
        f1 = f4
        ts.append(t)
        if done:
            break
        if nofailed:
            temp = 1.25 * (err / rtol) ** pow_
            if temp > 0.2:
                absh = absh / temp
            else:
                absh = 5.0 * absh
    if stats is not None:
        stats.update(steps=len(ts) - 1, failed=nfailed)
    return np.array(ts), y
