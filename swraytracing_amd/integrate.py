"""Packet integrators (L3): ode_symplectic and the qg-driver packet branch.

`ode_symplectic` keeps the reference signature (ode_symplectic.m:1).  With a
GPU-backed scheme (SpectralScheme / SnapshotPairScheme) the whole time loop
is one fused device pass (libswrt swrt_leapfrog: drift/kick/drift with the
packet in registers); any other RaytracingScheme runs the same Strang split
on the host through the scheme's U / grad_U_times_k (e.g. DifferenceScheme's
analytic callbacks).
"""
from __future__ import annotations

import math
import os

import numpy as np

from ._lib import Context, SwrtError
from .io import write_field
from .scheme import BUMP_QG, SnapshotPairScheme, SpectralScheme, flow_planes


def _omega(k, f, gH):
    return np.sqrt(f ** 2 + gH * np.sum(k * k, axis=1, keepdims=True))


def ode_symplectic(x0, k0, dt, T, f, gH, scheme):
    """[x, k, t] = ode_symplectic(x0, k0, dt, T, f, gH, scheme).

    x0, k0: 1 x 2 x P.  Returns x, k: Nsteps x 2 x P (row 1 = initial state)
    and t: (Nsteps,) with t(i) = (i-1)*dt (ode_symplectic.m:2-8,23-28)."""
    x0 = np.asarray(x0, dtype=np.float64)
    k0 = np.asarray(k0, dtype=np.float64)
    if x0.ndim == 2:
        x0 = x0[None]
        k0 = k0[None]
    P = x0.shape[2]
    Nsteps = int(math.floor(T / dt))
    x = np.zeros((Nsteps, 2, P))
    k = np.zeros((Nsteps, 2, P))
    t = np.arange(Nsteps, dtype=np.float64) * dt
    if Nsteps == 0:
        return x, k, t
    x[0] = x0[0]
    k[0] = k0[0]
    if Nsteps == 1:
        return x, k, t
    if isinstance(scheme, (SpectralScheme, SnapshotPairScheme)):
        nslots = 1 if isinstance(scheme, SpectralScheme) else 2
        xs = np.asfortranarray(x0[0].T)  # P x 2
        ks = np.asfortranarray(k0[0].T)
        _, _, hx, hk = scheme.ctx.leapfrog(xs, ks, dt, Nsteps - 1, f, gH, nslots=nslots, alpha0=0.0,
                                           dalpha=0.0, bump=scheme.bump, save_every=1)
        x[1:] = hx
        k[1:] = hk
        return x, k, t
    # generic host path (arbitrary RaytracingScheme)
    xc, kc = x0.copy(), k0.copy()

    def gv(kk):
        w = np.sqrt(f ** 2 + gH * (kk[:, 0:1, :] * kk[:, 0:1, :] + kk[:, 1:2, :] * kk[:, 1:2, :]))
        return gH * kk / w

    for i in range(1, Nsteps):
        x1 = xc + (dt / 2) * gv(kc)
        x2 = x1 + dt * scheme.U(x1)
        k2 = kc - dt * scheme.grad_U_times_k(x1, kc, 0)
        xc = x2 + (dt / 2) * gv(k2)
        kc = k2
        x[i] = xc[0]
        k[i] = kc[0]
    return x, k, t


def ode23_packets(ctx: Context, tspan, tmax, f, Cg, nslots=2, rtol=1e-3, atol=1e-6, bump=BUMP_QG,
                  allreduce_max=None, stats=None, controller=None, hook=None):
    """[~, y] = ode23(ray_ode, tspan, y0) for the device-resident packets
    (qgsw_raytrace.m:143-150, qg2layersw_raytrace.m:189-196): MATLAB ode23's
    Bogacki-Shampine controller (defaults RelTol 1e-3, AbsTol 1e-6, MaxStep
    0.1*|tspan|, max-norm error, its initial-step heuristic and step update)
    on the host, every per-packet stage on the GPU (swrt_ode23_*).  The error
    norm is global over all packets — with packets sharded over ranks pass
    ``allreduce_max`` (a callable max-reducing one float over the ranks, e.g.
    an RCCL all_reduce) so every rank takes the same steps.
    Parity: bit-identical to oracle ode23 (its restatement; MATLAB itself is
    unpinned).  Returns the accepted times.

    ``controller``: "library" runs this same controller inside the C library
    (swrt_ode23_run: no interpreter between attempts; with ``allreduce_max``
    swrt_ode23_run_sharded, which reduces stage 1's and every attempt's max
    through it), "python" the loop below (the one a rank without packets
    runs: the same reductions in the same order); default "library" for a
    Context.  Same steps and bits either way.

    ``hook``: a callable (QG calls only, never the packets) run once while
    the interval's first launches run — the library controller calls it
    after stage 1 and the first attempt are queued (swrt_ode23_run_hooked),
    the Python loop after stage 1."""
    if controller is None:
        controller = "library" if hasattr(ctx, "ode23_run") else "python"
    if controller == "library":
        try:
            ts, st = ctx.ode23_run(float(tspan[0]), float(tspan[1]), tmax, f, Cg, nslots, rtol, atol, bump,
                                   hook=hook, reduce=allreduce_max)
        except SwrtError as e:
            if "below hmin" in str(e):
                raise RuntimeError(str(e)) from e
            raise
        if stats is not None:
            stats.update(**st)
        return ts
    red = allreduce_max or (lambda v: v)
    t0, tfinal = float(tspan[0]), float(tspan[1])
    tdir = math.copysign(1.0, tfinal - t0)
    pw = 1.0 / 3.0
    rtol = max(rtol, 100 * np.finfo(float).eps)
    thr = atol / rtol
    htspan = abs(tfinal - t0)
    hmax = 0.1 * htspan
    t = t0
    rh = red(ctx.ode23_f1(t, tmax, f, Cg, nslots, thr, bump)) / (0.8 * rtol ** pw)
    if hook is not None:
        hook()
    absh = min(hmax, htspan)
    if absh * rh > 1:
        absh = 1.0 / rh
    absh = max(absh, 16 * np.spacing(t))
    ts = [t]
    done = False
    nfailed = 0
    attempts = 0
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
            tnew = t + h * 1.0
            if done:
                tnew = tfinal
            attempts += 1
            err = absh * red(ctx.ode23_attempt(t, h, tnew, tmax, f, Cg, nslots, thr, bump))
            h = tnew - t
            if err > rtol:
                nfailed += 1
                if absh <= hmin:
                    raise RuntimeError(f"ode23: step size {absh} below hmin at t={t}")
                if nofailed:
                    nofailed = False
                    absh = max(hmin, absh * max(0.5, 0.8 * (rtol / err) ** pw))
                else:
                    absh = max(hmin, 0.5 * absh)
                h = tdir * absh
                done = False
            else:
                break
        ctx.ode23_accept()
        t = tnew
        ts.append(t)
        if done:
            break
        if nofailed:
            temp = 1.25 * (err / rtol) ** pw
            absh = absh / temp if temp > 0.2 else 5.0 * absh
    if stats is not None:
        stats.update(steps=len(ts) - 1, failed=nfailed, attempts=attempts, accepted=len(ts))
    return np.array(ts)


class _EmptyShard:
    """The ode23 stages of a rank that holds no packets: every max is 0."""

    def ode23_f1(self, *a):
        return 0.0

    def ode23_attempt(self, *a):
        return 0.0

    def ode23_accept(self):
        pass


class PacketEnsemble:
    """Device-resident packets advanced through a sequence of background
    snapshots — the packet branch of qgsw_raytrace.m:140-163 /
    qg2layersw_raytrace.m:185-209 with the symplectic integrator instead of
    ode23.

    Per PDE step the caller hands the previous and current spectral PV
    (prev_qk, qk); grid_U runs on the GPU into slots 0/1 and the packets take
    `nsub` leapfrog substeps over [t, t+dt] with the kick of substep s at
    alpha = (s + 1/2)/nsub (interpolate_U's linear blend at the kick time).
    """

    def __init__(self, x, k, L, f, Cg, nx, K_d2, shear=0.0, k_scale=1.0, nlayers=1, device=0,
                 bump=BUMP_QG, ctx: Context | None = None, shard=None, bounds=None):
        """``shard`` = (rank, world): x, k are the whole ensemble (the same on
        every rank) and this rank advances its contiguous shard;
        frames are gathered to rank 0 on the device (dist.gather_packets) and
        ode23's error norm is max-reduced over the ranks.  ``bounds``: every
        rank's [lo, hi) (dist.shard_bounds / owner_bounds; default the even
        split).  A rank's shard may be empty (the PDE owner's, with weight 0):
        it then only takes part in the collectives."""
        self.ctx = ctx if ctx is not None else Context(device)
        self.L, self.f, self.Cg, self.nx = float(L), float(f), float(Cg), int(nx)
        self.gH = self.Cg ** 2
        self.K_d2, self.shear, self.k_scale = float(K_d2), float(shear), float(k_scale)
        self.ny_period = self.nx * nlayers
        self.bump = bump
        x = np.asarray(x, dtype=np.float64)
        k = np.asarray(k, dtype=np.float64)
        self.n_total = x.shape[0]
        self.rank, self.world = shard if shard is not None else (0, 1)
        self.bounds = None
        if self.world > 1:
            from .dist import shard_range
            self.bounds = list(bounds) if bounds is not None else \
                [shard_range(self.n_total, self.world, r) for r in range(self.world)]
            if len(self.bounds) != self.world or self.bounds[-1][1] != self.n_total:
                raise ValueError("bounds must give one [lo, hi) per rank covering the ensemble")
            lo, hi = self.bounds[self.rank]
            x, k = x[lo:hi], k[lo:hi]
        self.ctx.packets_set(x, k)
        self.n = x.shape[0]
        self._rebin = None

    def set_snapshots(self, prev_qk, qk):
        """grid_U(prev_qk) -> slot 0, grid_U(qk) -> slot 1 (layer 1 if 3-D)."""
        for slot, q in enumerate((prev_qk, qk)):
            q = np.asarray(q, dtype=np.complex128)
            if q.ndim == 3:
                q = q[:, :, 0]
            self.ctx.set_field_qk(slot, q, self.nx, self.L, self.K_d2, self.shear, self.k_scale,
                                  self.ny_period)

    def set_grid_snapshots(self, flow1, flow2):
        for slot, fl in enumerate((flow1, flow2)):
            self.ctx.set_field_grid(slot, flow_planes(fl), self.nx, self.L, self.ny_period)

    def advance(self, dt, nsub=1, save_every=0):
        if self.n == 0:
            return
        # re-bin after ~4 PDE intervals of packet motion: every 4 steps at one
        # substep per interval, every 20 at five (tuned on the bench workload)
        if self._rebin != 4 * nsub:
            self._rebin = 4 * nsub
            self.ctx.set_locality(self._rebin, 0)
        h = dt / nsub
        self.ctx.advance(h, nsub, self.f, self.gH, nslots=2, alpha0=0.5 / nsub, dalpha=1.0 / nsub,
                         bump=self.bump, save_every=save_every)

    def advance_intervals(self, dts, nsub=1, save_every=0):
        """len(dts) consecutive PDE intervals in one call, interval i between
        the snapshots in slots i and i+1 (swrt_advance_intervals): the same
        bits as one advance() per interval with the pair moved to slots 0, 1."""
        if self.n == 0:
            return
        if self._rebin != 4 * nsub:
            self._rebin = 4 * nsub
            self.ctx.set_locality(self._rebin, 0)
        self.ctx.advance_intervals([dt / nsub for dt in dts], nsub, self.f, self.gH, alpha0=0.5 / nsub,
                                   dalpha=1.0 / nsub, bump=self.bump, save_every=save_every)

    def advance_ode23(self, dt, rtol=1e-3, atol=1e-6, allreduce_max=None, stats=None, controller=None, hook=None):
        """The reference drivers' own integrator over [0, dt] with
        interpolate_U's alpha = t/dt (ode23(ray_ode, [0, dt], y0));
        ``controller`` and ``hook`` as in ode23_packets."""
        if allreduce_max is None and self.world > 1:
            import torch.distributed as dist

            from .dist import allreduce_max_fn
            allreduce_max = allreduce_max_fn(backend=dist.get_backend())
        # an empty shard contributes 0 to every error max (the max-norm's identity)
        ctx = self.ctx if self.n > 0 else _EmptyShard()
        return ode23_packets(ctx, (0.0, dt), dt, self.f, self.Cg, nslots=2, rtol=rtol, atol=atol,
                             bump=self.bump, allreduce_max=allreduce_max, stats=stats, controller=controller,
                             hook=hook)

    def state(self):
        return self.ctx.packets_get()

    def write_frame(self, t, directory):
        """qgsw_raytrace.m:159-162: wrapped x, k and t appended to
        packet_x.bin / packet_k.bin / packet_time.bin.  Sharded: a collective
        (every rank calls it); rank 0 writes the whole ensemble."""
        if self.world > 1:
            from .dist import gather_packets
            full = gather_packets(self.ctx, self.n_total, self.world, self.rank, bounds=self.bounds)
            if full is None:
                return
            x, k = full
        else:
            x, k = self.state()
        L = self.L
        write_field(np.mod(x + L / 2, L) - L / 2, os.path.join(directory, "packet_x"))
        write_field(k, os.path.join(directory, "packet_k"))
        write_field(np.array([[t]]), os.path.join(directory, "packet_time"))


def step_packet_xka(P, U, GradU, H, C0, f, dx, dy, dt, nsteps=1, ctx: Context | None = None):
    """Pout = step_packet_xka(P, U, GradU, H, C0, f, dx, dy, dt)
    (ray_trace_sw/step_packet_xka.m:1-91) on the GPU.

    P: dict with x, y, k, l, a (scalars or equal-length arrays = many packets).
    U: dict u, v; GradU: dict u_x, u_y, v_x, v_y; H: field (nx x nx).
    `nsteps` > 1 repeats the step (the raytrace_sw.m:125-130 loop) on device."""
    from .scheme import default_context
    ctx = ctx or default_context()
    if not np.allclose(np.asarray(H).shape, np.asarray(U["u"]).shape) or np.asarray(H).shape[0] != np.asarray(H).shape[1]:
        raise ValueError("fields must be nx x nx")
    ctx.xka_set_fields(U, GradU, H, dx, dy)
    names = ("x", "y", "k", "l", "a")
    scalar = np.ndim(P["x"]) == 0
    st = np.stack([np.atleast_1d(np.asarray(P[n], dtype=np.float64)) for n in names], axis=1)
    out, _ = ctx.xka_step(st, C0, f, dt, nsteps)
    return {n: (float(out[0, i]) if scalar else out[:, i].copy()) for i, n in enumerate(names)}


def raytrace_xka(P0, U, GradU, H, C0, f, dx, dy, dt, nsteps, ctx: Context | None = None):
    """The packet loop of ray_trace_sw/raytrace_sw.m:124-130: P(i, 1) = P0(i),
    P(i, j) = step_packet_xka(P(i, j-1), ...) for j = 2..nsteps.  Returns a dict
    of (np, nsteps) arrays (column j-1 = state after j-1 steps)."""
    from .scheme import default_context
    ctx = ctx or default_context()
    ctx.xka_set_fields(U, GradU, H, dx, dy)
    return _trace_xka(ctx, P0, C0, f, dt, nsteps)


def rsw_background(S, f, Cg, L=2 * np.pi, ctx: Context | None = None):
    """U, GradU, H of ray_trace_sw/raytrace_sw.m:16-52 from an RSW state
    S = [u v eta] (nx x nx x 3): the geostrophic projection and its seven
    k2g run on the GPU, and the result stays there as the xka background
    (the next raytrace_sw / step_packet_xka call on ctx uses it without a
    re-upload).  Returns host copies (U dict, GradU dict, H)."""
    from .scheme import default_context
    ctx = ctx or default_context()
    ctx.xka_set_rsw(S, f, Cg, L)
    return ctx.xka_get_fields()


def raytrace_sw(S, f, Cg, P0, dt, nsteps, L=2 * np.pi, ctx: Context | None = None):
    """ray_trace_sw/raytrace_sw.m end to end on the GPU: the background of
    :16-52 from S = [u v eta], then the packet loop of :124-130 with
    step_packet_xka(P, U, GradU, H, C0 = Cg, f, dx, dx, dt) (:22-23, 130).
    Returns the (np, nsteps) dict of raytrace_xka."""
    from .scheme import default_context
    ctx = ctx or default_context()
    ctx.xka_set_rsw(S, f, Cg, L)
    return _trace_xka(ctx, P0, Cg, f, dt, nsteps)


def _trace_xka(ctx, P0, C0, f, dt, nsteps):
    names = ("x", "y", "k", "l", "a")
    st = np.stack([np.atleast_1d(np.asarray(P0[n], dtype=np.float64)) for n in names], axis=1)
    npk = st.shape[0]
    out = {n: np.zeros((npk, nsteps)) for n in names}
    for i, n in enumerate(names):
        out[n][:, 0] = st[:, i]
    if nsteps > 1:
        _, hist = ctx.xka_step(st, C0, f, dt, nsteps - 1, save_every=1)
        for i, n in enumerate(names):
            out[n][:, 1:] = hist[:, :, i].T
    return out
