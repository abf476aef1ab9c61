"""The QG PDE steppers that produce the packets' background snapshots, with
their state resident on the GPU, and the two reference
drivers built on them.

* :class:`QGModel` — ``qgsw_raytrace.m:111-137`` (1 layer: AB3 + filter,
  ``update`` :270-286) and ``qg2layersw_raytrace.m:129-181`` (2 layers:
  exponential AB3, adaptive CFL :156-165) over ``swrt_qg_*``.
* :func:`qgsw_raytrace` / :func:`qg2layersw_raytrace` — the drivers
  (``qgsw_raytrace.m:1-180``, ``qg2layersw_raytrace.m:1-247``): PDE on the
  device, per PDE step grid_U of (prev_qk, qk) straight into the packet slots
  and the packets advanced through [t, t+dt] by the fused symplectic kernel
  (the reference's ``ode23`` is replaced by ``nsub`` leapfrog substeps with the
  interpolate_U blend), frames written in the reference's
  ``data/*.bin`` layout (``write_field.m``).
"""
from __future__ import annotations

import math
import os

import numpy as np

from ._lib import Context, QGParams
from .integrate import PacketEnsemble
from .io import write_field
from .runlog import RunLog, parameter_block
from .scheme import BUMP_QG


class QGModel:
    """Device-resident spectral QG model (``swrt_qg_init`` / ``swrt_qg_step``).

    ``qk``: the g2k half plane, (2kmax+1, kmax+1) for one layer or
    (2kmax+1, kmax+1, 2) for two."""

    def __init__(self, qk, nx, params: QGParams, ctx: Context | None = None, device=0):
        self.ctx = ctx if ctx is not None else Context(device)
        self.nx = int(nx)
        self.params = params
        self.nlayers = params.nlayers
        self.L = params.L
        self.dx = params.L / nx
        self.spec_pending = False  # a speculative step is queued (step_speculative) and not yet resolved
        self.ctx.qg_init(params, nx, qk)

    @classmethod
    def one_layer(cls, qk, nx, f, Cg, beta=0.0, r_drag=0.1, force_strength=0.1, use_filter=True, **kw):
        """qgsw_raytrace.m:22-27,111-137: L = 2*pi, K_d2 = f/Cg, inertial_ring forcing."""
        p = QGParams(nlayers=1, filter=1 if use_filter else 0, L=2 * math.pi, K_d2=f / Cg, beta=beta,
                     r_drag=r_drag, force_strength=force_strength, f=f, Cg=Cg, shear=0.0, nu=0.0,
                     hyper_order=0.0, r=0.0)
        return cls(qk, nx, p, **kw)

    @classmethod
    def two_layer(cls, qk, nx, f, Cg, L=20.0, beta=0.0, shear=0.5, alpha=4, r=0.4, nutune=0.1, **kw):
        """qg2layersw_raytrace.m:13-34,79,129-147."""
        dx = L / nx
        p = QGParams(nlayers=2, filter=0, L=L, K_d2=f / Cg, beta=beta, r_drag=0.0, force_strength=0.0, f=f,
                     Cg=Cg, shear=shear, nu=nutune * dx ** (2 * alpha), hyper_order=float(alpha), r=r)
        return cls(qk, nx, p, **kw)

    def settle(self):
        """Drop a pending speculative step (the model stays at the committed
        step).  The calls the library refuses while one is pending — step,
        max_speed(_async), snapshot — settle first, so code that touches the
        model after a TwoLayerLoop never meets SWRT_ERR_STATE."""
        if self.spec_pending:
            self.resolve(False)

    def step(self, dt, nsteps=1):
        self.settle()
        self.ctx.qg_step(dt, nsteps)

    def step_speculative(self, dt):
        """Queue the next step with dt and its CFL read-back before the current
        U0 is known; the committed state stays until resolve()."""
        self.ctx.qg_step_speculative(dt)
        self.spec_pending = True

    def resolve(self, accept):
        self.ctx.qg_resolve(accept)
        self.spec_pending = False

    def max_speed(self):
        """U0 = sqrt(max(u.^2 + v.^2)) of grid_U(qk) (all layers, u + shear)."""
        self.settle()
        return self.ctx.qg_max_speed()

    def cfl_rule(self, dt, U0, cfl_fraction):
        """qg2layersw_raytrace.m:159-165 given U0: returns (dt, changed)."""
        cond = cfl_fraction * self.dx / U0
        if cond < dt or dt < cond / 4:
            return cfl_fraction / 2 * self.dx / U0, True
        return dt, False

    def cfl_update(self, dt, cfl_fraction):
        """qg2layersw_raytrace.m:156-165: returns (dt, U0, changed)."""
        U0 = self.max_speed()
        dt, changed = self.cfl_rule(dt, U0, cfl_fraction)
        return dt, U0, changed

    def max_speed_async(self):
        """Enqueue U0 of the current qk; collect it with max_speed_result()
        after queueing other work (the driver queues the packets first)."""
        self.settle()
        self.ctx.qg_max_speed_async()

    def max_speed_result(self):
        return self.ctx.qg_max_speed_result()

    @property
    def qk(self):
        return self.ctx.qg_get()[0]

    @property
    def t(self):
        return self.ctx.qg_get()[1]

    @property
    def steps(self):
        return self.ctx.qg_get()[2]

    def q(self):
        """k2g(qk) per layer: (nx, nx) or (nx, nx, 2)."""
        q = self.ctx.qg_get_q()
        return q[:, :, 0] if self.nlayers == 1 else q

    def snapshot(self, slot, which=0, layer=0, ny_period=0):
        """grid_U of the current (0) / previous (1) qk into packet slot `slot`."""
        self.settle()
        self.ctx.qg_snapshot(slot, which, layer, ny_period)

    def snapshot_speculative(self, slot, ny_period=0):
        """Layer 0's grid_U of the pending speculative step into `slot`: the
        snapshot(slot) this step gives once accepted (bit for bit)."""
        self.ctx.qg_snapshot_speculative(slot, ny_period)


# ----------------------------------------------------------------------------
# Drivers
# ----------------------------------------------------------------------------
def initial_q(nx, L, a_g, K_d2, k_min, k_max, rng, ndgrid=False):
    """initial_q (qgsw_raytrace.m:191-214, qg2layersw_raytrace.m:258-281): a
    random-phase ring k_min < |k| <= k_max normalised to max|U| = a_g, on
    linspace(-L/2, L/2, nx) (meshgrid for 1 layer, ndgrid for 2).  numpy's
    generator replaces MATLAB's rng (its stream is not reproducible here)."""
    xs = np.linspace(-L / 2, L / 2, nx)
    X, Y = np.meshgrid(xs, xs, indexing="ij" if ndgrid else "xy")
    q = np.zeros_like(X)
    U = np.zeros_like(X)
    V = np.zeros_like(X)
    phase = 2 * np.pi * rng.random((2 * k_max + 1, 2 * k_max + 1))
    for k in range(-k_max, k_max + 1):
        for l in range(-k_max, k_max + 1):
            if k_min ** 2 < k * k + l * l <= k_max ** 2:
                wp = k * X + l * Y + phase[k + k_max, l + k_max]
                U = U - l * np.sin(wp)
                V = V + k * np.sin(wp)
                q = q - (K_d2 + k * k + l * l) * np.cos(wp)
    return a_g / np.sqrt((U ** 2 + V ** 2).max()) * q


def _packets(N, L, near_inertial_factor, f, Cg, rng):
    """qgsw_raytrace.m:54-60."""
    wf = math.sqrt((near_inertial_factor ** 2 - 1) * f ** 2 / Cg ** 2)
    i = np.arange(1, N + 1, dtype=np.float64)
    k = np.stack([wf * np.cos(2 * np.pi * i / N), wf * np.sin(2 * np.pi * i / N)], axis=1)
    x = L * rng.random((N, 2)) - L / 2
    return x, k


class _IntervalGroup:
    """Packet intervals deferred until `k` PDE steps have their end snapshots
    (slots 1..k; slot 0 holds the group's start), then advanced in one
    swrt_advance_intervals call — the same bits as one advance per step.  The
    PDE runs up to k steps ahead of the packets; a frame write flushes."""

    def __init__(self, ctx, ens, k, nsub, integrator="leapfrog"):
        if integrator not in ("leapfrog", "ode23"):
            raise ValueError("integrator must be 'leapfrog' or 'ode23'")
        self.ctx, self.ens, self.nsub, self.integrator = ctx, ens, nsub, integrator
        # ode23 (the reference's own packet integrator) takes one interval per call
        self.k = 1 if integrator == "ode23" else max(1, min(int(k), 4))
        self.dts = []
        # ode23 controller totals over the calls (steps, failed, attempts)
        self.ode23_stats = {"steps": 0, "failed": 0, "attempts": 0, "intervals": 0}

    def next_slot(self):
        return len(self.dts) + 1

    def add(self, dt, hook=None):
        """hook (ode23 only): run while the interval's first launches run."""
        self.dts.append(dt)
        if len(self.dts) == self.k:
            self.flush(hook)
        elif hook is not None:
            hook()

    def flush(self, hook=None):
        if self.dts:
            if self.integrator == "ode23":
                st = {}
                # ode23(ray_ode, [0, dt], y0), alpha = t/dt
                self.ens.advance_ode23(self.dts[0], stats=st, hook=hook)
                for key in ("steps", "failed", "attempts"):
                    self.ode23_stats[key] += int(st.get(key, 0))
                self.ode23_stats["intervals"] += 1
            else:
                self.ens.advance_intervals(self.dts, self.nsub)
                if hook is not None:
                    hook()
            self.ctx.swap_slots(0, len(self.dts))  # the last end snapshot starts the next group
            self.dts = []


def _dist_info():
    """(rank, world) of an initialised torch.distributed job, else (0, 1)."""
    try:
        import torch.distributed as dist
    except ImportError:
        return 0, 1
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _fresh_outputs(out_dir, fresh):
    """write_field.m:31 appends to existing files; a driver run starting from
    t = 0 removes earlier outputs first unless fresh=False."""
    os.makedirs(out_dir, exist_ok=True)
    if not fresh:
        return
    for name in ("packet_x", "packet_k", "packet_time", "pv", "pv_time"):
        p = os.path.join(out_dir, name + ".bin")
        if os.path.exists(p):
            os.remove(p)


def _owner_setup(world, pde, owner_weight, nx, Npackets, link_buffers="auto"):
    """(link, bounds) of a sharded run in the PDE-owner form, or (None, None)
    for the replicated form (every rank steps the PDE).  link_buffers: "auto"
    (device buffers with nccl, host buffers with gloo), "device" or "host"."""
    if world <= 1 or pde == "replicated":
        return None, None
    if pde != "owner":
        raise ValueError("pde must be 'owner' or 'replicated'")
    import torch.distributed as dist

    from .dist import OwnerLink, owner_bounds
    device = {"auto": None, "device": True, "host": False}[link_buffers]
    w0 = owner_weight_for(world) if owner_weight is None else owner_weight
    return OwnerLink(nx, dist.get_backend(), device=device), owner_bounds(Npackets, world, w0)


def owner_weight_for(world):
    """The PDE owner's packets per packet of a receiving rank, from the
    measured one-GPU legs of bench.py's driver_step_forecast["owner"]
    (profiles/r06_final): with 2 ranks the owner's PDE leaves room for
    packets (best w = 0.5), from 4 ranks on the receivers' share is what
    bounds the step and the owner's PDE already takes about as long as it
    (best w = 0: the owner holds no packets)."""
    return 0.5 if world <= 2 else 0.0


class TwoLayerLoop:
    """One iteration of qg2layersw_raytrace.m:152-197 on the device: the CFL
    rule (:156-165) on the current U0, the PDE step, U0 of the new qk read back
    asynchronously (collected after the packet work is queued, so the rule
    never idles the GPU), and — once t > packet_delay — grid_U of (prev_qk,
    qk) into the packet slots and the packet interval [t, t+dt].  Used by
    :func:`qg2layersw_raytrace` (which adds the frame writes) and by bench.py's
    end-to-end driver-step figure.

    With ``speculate`` (default) every step returns with the next PDE step
    queued speculatively (QGModel.spec_pending); the model's own calls drop
    it before they run (QGModel.settle), and :meth:`settle` does so explicitly.

    ``link`` (dist.OwnerLink): this rank is the PDE owner of a sharded run —
    after each PDE step it publishes the new qk's top layer and dt to the
    other ranks (:class:`ReceiverLoop`), which build their snapshots from it."""

    SPEC_SLOT = 2  # ode23 + speculate: where the next step's snapshot is packed ahead (slots 0/1: the interval's)

    def __init__(self, model, ens, dt, U0, cfl_fraction=0.25, packet_delay=0.0, nsub=5, packet_intervals=1,
                 integrator="leapfrog", log=None, speculate=True, link=None):
        self.model, self.ens, self.dt, self.U0 = model, ens, dt, U0
        self.link = link
        # speculate: each step also queues the NEXT PDE step with this step's
        # dt (swrt_qg_step_speculative) before waiting for this step's U0, so
        # the QG stream never idles through the host's read-back and CFL rule;
        # the rule then accepts it, or drops it and steps with its new dt —
        # the same computation either way (bit-identical files)
        self.speculate = speculate
        self.cfl_fraction, self.packet_delay = cfl_fraction, packet_delay
        self.nx = model.nx
        self.t = 0.0
        self.steps = 0
        self.dts = []
        self.have_cur = False
        self.log = log
        self.group = _IntervalGroup(model.ctx, ens, packet_intervals, nsub, integrator) if ens is not None else None
        # ode23 with speculation: the speculative step's snapshot is packed into
        # slot SPEC_SLOT while the interval runs; an accepted step takes it by
        # a slot swap instead of a snapshot launch between the intervals
        self._spec_snap = False
        # ode23 + speculate: chain each interval's stage 1 to the previous call
        # (swrt_ode23_chain_next; SWRT_ODE23_CHAIN=0 turns it off for A/B runs)
        self.chain = os.environ.get("SWRT_ODE23_CHAIN", "1") != "0"

    def step(self):
        """Returns True when the packets advanced through this PDE step."""
        self.steps += 1
        self.dt, changed = self.model.cfl_rule(self.dt, self.U0, self.cfl_fraction)
        if changed and self.log is not None:
            self.log(f"CFL condition not met, max|u|={self.U0:f}, new dt={self.dt:f}\n")
        self.dts.append(self.dt)
        if self.model.spec_pending:
            # the step queued by the previous call with the previous dt
            self.model.resolve(not changed)
            if changed:
                self.model.step(self.dt)
                self.model.max_speed_async()
        else:
            self.model.step(self.dt)
            self.model.max_speed_async()
        self.t = self.t + self.dt
        active = self.ens is not None and self.t > self.packet_delay
        spec = self.speculate and self.model.params.nlayers == 2 and getattr(self.model.ctx, "qg_fused", True)
        # ode23 intervals of a sharded run hold collectives (the error norm's
        # allreduce per attempt): the owner publishes before its interval, as
        # the receivers need this step's qk before theirs
        publish_first = self.link is not None and self.group is not None and self.group.integrator == "ode23"
        if publish_first:
            self.link.publish(self.model.ctx, self.dt)
        if active and self.ens.n == 0:
            # an owner without packets: no snapshots; the interval still runs
            # (ode23: its error-norm collectives) with the speculative step inside
            if spec and self.group.integrator == "ode23":
                dt = self.dt
                self.group.add(dt, hook=lambda: self.model.step_speculative(dt))
                spec = False
            else:
                self.group.add(self.dt)
        elif active:
            ny = 2 * self.nx
            if not self.have_cur:
                self.model.snapshot(0, which=1, layer=0, ny_period=ny)
            if self._spec_snap and not changed and self.have_cur:
                # this (accepted) step's snapshot, packed during the last interval
                self.model.ctx.swap_slots(self.group.next_slot(), self.SPEC_SLOT)
            else:
                self.model.snapshot(self.group.next_slot(), which=0, layer=0, ny_period=ny)
            self._spec_snap = False
            self.have_cur = True
            if spec and self.group.integrator == "ode23":
                # the ode23 interval holds the host until it ends (its step-size
                # controller), so the next PDE step — and its snapshot — are
                # queued from inside it, once its first launches are queued
                # (swrt_ode23_run_hooked), and run beside its attempts; the
                # leapfrog interval only queues work and returns
                dt = self.dt

                def hook():
                    self.model.step_speculative(dt)
                    self.model.snapshot_speculative(self.SPEC_SLOT, ny_period=ny)
                    self._spec_snap = True
                    if self.chain:  # (sharded too: swrt_ode23_run_sharded takes a chained stage 1)
                        # the next interval reads this one's end snapshot (slot
                        # 1) and the one just queued: its stage 1 is queued as
                        # this interval ends (taken only if still exact)
                        self.model.ctx.ode23_chain_next(1, self.SPEC_SLOT)
                self.group.add(dt, hook=hook)
                spec = False
            else:
                self.group.add(self.dt)
        else:
            self.have_cur = False
            self._spec_snap = False
        if spec:
            self.model.step_speculative(self.dt)
        if self.link is not None and not publish_first:
            # this step's committed qk to the other ranks: queued after the
            # next (speculative) step, so its host calls are off the PDE's
            # critical path (U0 read-back -> CFL rule -> next step)
            self.link.publish(self.model.ctx, self.dt)
        self.U0 = self.model.max_speed_result()  # this step's (read-backs pop oldest first)
        return active

    def flush(self):
        if self.group is not None:
            self.group.flush()

    def settle(self):
        """Drop a pending speculative step: the model stays at the committed
        step.  Optional: QGModel's step / max_speed / snapshot settle on their
        own, so PDE calls after the loop need no explicit settle."""
        self.model.settle()


class ReceiverLoop:
    """A receiving rank's iteration of qg2layersw_raytrace.m:152-197 in the
    PDE-owner form of a sharded run: no PDE here — the owner's dt and the
    new qk's top layer arrive through ``link`` (dist.OwnerLink) each step,
    grid_U of it (and, on the first active step, of the previous qk) goes
    into the packet slots (swrt_snapshot_qk: the owner's snapshot bits), and
    this rank's packets take the interval [t, t+dt] exactly as the owner's
    TwoLayerLoop does (same t, dt sequence, active steps and frame points)."""

    def __init__(self, link, ens, dt, packet_delay=0.0, nsub=5, packet_intervals=1, integrator="leapfrog",
                 ahead=None):
        self.link, self.ens, self.dt = link, ens, dt
        self.packet_delay = packet_delay
        self.t = 0.0
        self.steps = 0
        self.dts = []
        self.have_cur = False
        self.group = _IntervalGroup(ens.ctx, ens, packet_intervals, nsub, integrator) if ens is not None else None
        # The host queues step n only once the packet work of step n - ahead
        # has finished.  Unpaced, a receiver whose packets are slower than the
        # owner's PDE queues snapshots until every spare slot buffer still
        # looks in use; the next snapshot then waits for the packet launch
        # before it and packets and snapshots run one after the other
        # (swrt_qg_snapshot's renaming decides at queue time).
        # the mark is an event recorded after every 2nd step's packet work (an
        # event between two kernels costs ~6 us of idle GPU, tools/owner_legs.py
        # traces), so the host is `ahead` to `ahead` + 1 steps ahead
        self.mark_every = 2
        nbuf = getattr(link, "nbuf", 2)
        self.ahead = (nbuf - self.mark_every - 1) if ahead is None else int(ahead)
        self._done = []  # (step, event)
        self._pk = None
        if self.ahead > 0 and ens is not None and ens.n > 0 and getattr(link, "device", False):
            import torch
            self._pk = torch.cuda.ExternalStream(ens.ctx.stream())
            self._events = [torch.cuda.Event() for _ in range(self.ahead + 2)]
            self._ev_i = 0
        # device link with pacing: the host waits for each broadcast and the
        # pacing orders the buffers' refills, so the snapshots need no
        # cross-stream events (OwnerLink.snapshot fenced): the buffer of step m
        # is read by step m's snapshot and, on a first active step, by step
        # m + 1's grid_U(prev_qk); it is refilled by receive m + nbuf, by which
        # the host has waited for the packet work of step m + nbuf - ahead -
        # mark_every or later — after both reads when that is >= m + 1
        self._fenced = self._pk is not None and self.ahead + self.mark_every + 1 <= nbuf

    def _snapshot(self, slot, which):
        e = self.ens
        self.link.snapshot(e.ctx, slot, which, e.L, e.K_d2, e.shear, e.k_scale, e.ny_period, fenced=self._fenced)

    def step(self):
        self.steps += 1
        while self._done and self._done[0][0] <= self.steps - 1 - self.ahead:
            self._done.pop(0)[1].synchronize()
        self.dt = self.link.receive(wait=self._fenced)
        self.dts.append(self.dt)
        self.t = self.t + self.dt
        active = self.ens is not None and self.t > self.packet_delay
        if active:
            if self.ens.n > 0:
                if not self.have_cur:
                    self._snapshot(0, 1)  # grid_U(prev_qk)
                self._snapshot(self.group.next_slot(), 0)  # grid_U(qk)
                self.have_cur = True
            self.group.add(self.dt)
            if self._pk is not None and self.steps % self.mark_every == 0:
                ev = self._events[self._ev_i]
                self._ev_i = (self._ev_i + 1) % len(self._events)
                ev.record(self._pk)
                self._done.append((self.steps, ev))
        else:
            self.have_cur = False
        return active

    def flush(self):
        if self.group is not None:
            self.group.flush()

    def settle(self):
        pass


def qgsw_raytrace(nx, Npackets, near_inertial_factor, T_Fr_days, packet_delay_days, U_g, f, Cg, *,
                  out_dir="data", nsub=4, max_steps=None, seed=146, verbose=False, r_drag=0.1,
                  packet_intervals=1, integrator="leapfrog", fresh=True, ctx: Context | None = None,
                  pde="owner", owner_weight=None, link_buffers="auto"):
    """qgsw_raytrace.m:1-180 with the PDE and the packets on the GPU.

    Writes ``out_dir``/packet_x.bin, packet_k.bin, packet_time.bin, pv.bin,
    pv_time.bin (frames appended, write_field.m) and run.log.  ``max_steps``
    bounds the run (None: the reference's Nsteps = ceil(T/dt)).  ``r_drag``
    (0.1 in the reference, :25) enters update as the literal `+ r_drag*K2`
    term of :285, which forces every mode and makes long runs blow up; pass
    0 to drop it.  ``packet_intervals`` (1..4): PDE steps whose packet
    intervals go to the device in one call (results identical for any
    value; 1 is faster end to end here: the PDE chain's latency, not the
    packet launch, bounds a driver step).  ``integrator``:
    "leapfrog" (``nsub`` fused symplectic substeps per PDE interval) or
    "ode23" (the reference's own ode23 over each interval, qgsw_raytrace.m:149).
    ``fresh``: remove earlier output files first (default) or append to
    them as write_field.m:31 does.  ``pde``, ``owner_weight``: the sharded
    forms, as in :func:`qg2layersw_raytrace`.  Returns a dict of run facts
    (dt, Nsteps, steps run, frames written, final t)."""
    ctx = ctx if ctx is not None else Context(0)
    timing = getattr(ctx, "timing_every", 1)
    ctx.set_timing(0)  # (no HIP-event pair around every packet launch; restored at the end)
    rank, world = _dist_info()  # sharded run: packets split over the ranks
    if rank == 0:
        _fresh_outputs(out_dir, fresh)
    log = RunLog(os.path.join(out_dir, "run.log") if rank == 0 else None, verbose and rank == 0)
    L = 2 * math.pi
    dx = L / nx
    rng = np.random.default_rng(seed)
    K_d2 = f / Cg
    T_days = T_Fr_days / f
    CFL_fraction = 0.05
    steps_per_save = 50
    packet_delay = packet_delay_days / f
    packet_steps_per_save = 5
    q = initial_q(nx, L, U_g, K_d2, 5, 8, rng)
    qk = ctx.g2k(q)
    x, k = _packets(Npackets, L, near_inertial_factor, f, Cg, rng)
    model = QGModel.one_layer(qk, nx, f, Cg, r_drag=r_drag, ctx=ctx)
    link, bounds = _owner_setup(world, pde, owner_weight, nx, Npackets, link_buffers)
    if link is not None:
        link.seed(ctx)
    owner = link is None or rank == 0  # this rank steps the PDE
    if link is not None and owner:
        link.bind_owner(ctx)
    if not owner:
        ctx.qg_set_stream(False)  # (snapshots in series with the packets, as in qg2layersw_raytrace)
        ctx.set_packet_streams(1)
    U0 = model.max_speed()
    Fr = U0 / Cg
    T = T_days / Fr ** 2
    dt = CFL_fraction * dx / U0
    Nsteps = math.ceil(T / dt)
    packet_step_start = math.ceil(packet_delay / dt)
    log(parameter_block(nx, Npackets, near_inertial_factor * f, dt, T, packet_delay, steps_per_save,
                        packet_steps_per_save, f, Cg, U_g, U0, Fr, K_d2))
    ens = PacketEnsemble(x, k, L, f, Cg, nx, K_d2, shear=0.0, k_scale=1.0, nlayers=1, bump=BUMP_QG, ctx=ctx,
                         shard=(rank, world), bounds=bounds) \
        if Npackets > 0 else None

    def snapshot(slot, which):
        if owner:
            model.snapshot(slot, which=which)
        else:
            link.snapshot(ctx, slot, which, L, K_d2, 0.0, 1.0, 0)
    t = 0.0
    frames = 1
    if ens is not None:
        ens.write_frame(dt * (packet_step_start - 1), out_dir)
    if rank == 0:
        write_field(model.q(), os.path.join(out_dir, "pv"))
        write_field(np.array([[t]]), os.path.join(out_dir, "pv_time"))
    nrun = Nsteps if max_steps is None else min(Nsteps, int(max_steps))
    have_cur = False
    group = _IntervalGroup(ctx, ens, packet_intervals, nsub, integrator) if ens is not None else None
    log.start()
    for step in range(1, nrun + 1):
        if owner:
            model.step(dt)
            if link is not None:
                link.publish(ctx, dt)
        else:
            link.receive()  # (the 1-layer driver's dt is fixed)
        t = t + dt
        if ens is not None and t > packet_delay:
            if ens.n > 0:
                if not have_cur:
                    snapshot(0, 1)  # grid_U(prev_qk); later groups start from the last grid_U(qk)
                snapshot(group.next_slot(), 0)  # grid_U(qk)
            have_cur = True
            group.add(dt)
            if (step - packet_step_start + 1) % packet_steps_per_save == 0:
                group.flush()
                ens.write_frame(t, out_dir)
                frames += 1
        else:
            have_cur = False
        if step % steps_per_save == 0 and rank == 0:
            write_field(model.q(), os.path.join(out_dir, "pv"))
            write_field(np.array([[t]]), os.path.join(out_dir, "pv_time"))
        log.progress(step, Nsteps)
    if group is not None:
        group.flush()
    if link is not None:
        link.close()
    ctx.synchronize()
    ctx.set_timing(timing)
    log.finish()
    log.close()
    return dict(dt=dt, Nsteps=Nsteps, steps=nrun, packet_frames=frames, t=t, U0=U0,
                packet_step_start=packet_step_start)


def qg2layersw_raytrace(nx, Npackets, near_inertial_factor, T_Fr_days, packet_delay_Fr_days, U_g, f, Cg, *,
                        out_dir="data", nsub=5, max_steps=None, seed=5, verbose=False,
                        packet_intervals=1, integrator="leapfrog", fresh=True, ctx: Context | None = None,
                        pde="owner", owner_weight=None, link_buffers="auto"):
    """qg2layersw_raytrace.m:1-247 with the PDE and the packets on the GPU
    (adaptive CFL :156-165, packets on layer 1 with u += shear_strength and
    interpolate's 2*nx y-period).  Same packet outputs as :func:`qgsw_raytrace`;
    pv.bin holds the initial nx x nx x 2 frame only, as in the reference.
    ``packet_intervals``, ``integrator``, ``fresh``: as in :func:`qgsw_raytrace`.

    Sharded (torch.distributed, world > 1): ``pde="owner"`` (default) — rank 0
    steps the PDE and sends each step's top-layer qk and dt to the other
    ranks, which only build snapshots and advance packets; rank 0 holds
    ``owner_weight`` packets per packet of another rank (dist.owner_bounds;
    default owner_weight_for(world)).
    ``pde="replicated"``: every rank steps the same PDE, packets split evenly.
    Both write the single-process files byte for byte.  ``link_buffers``: the
    owner link's buffers ("auto": on the device with nccl, on the host with
    gloo; "device" / "host" to force one)."""
    ctx = ctx if ctx is not None else Context(0)
    timing = getattr(ctx, "timing_every", 1)
    ctx.set_timing(0)  # (no HIP-event pair around every packet launch; restored at the end)
    rank, world = _dist_info()  # sharded run: packets split over the ranks
    if rank == 0:
        _fresh_outputs(out_dir, fresh)
    log = RunLog(os.path.join(out_dir, "run.log") if rank == 0 else None, verbose and rank == 0)
    L = 20.0
    dx = L / nx
    rng = np.random.default_rng(seed)
    K_d2 = f / Cg
    shear = 0.5
    T_Fr = T_Fr_days / f
    packet_delay_Fr = packet_delay_Fr_days / f
    CFL_fraction = 0.25
    steps_per_save = 10
    packet_delay_steps = packet_delay_Fr / f
    packet_steps_per_save = 25
    q1 = initial_q(nx, L, U_g, K_d2, 10, 30, rng, ndgrid=True)
    qk1 = ctx.g2k(q1)
    qk2 = ctx.g2k(-q1)
    qk = np.stack([qk1, qk2], axis=2)
    x, k = _packets(Npackets, L, near_inertial_factor, f, Cg, rng)
    model = QGModel.two_layer(qk, nx, f, Cg, L=L, shear=shear, ctx=ctx)  # (every rank: the same U0, T, dt)
    link, bounds = _owner_setup(world, pde, owner_weight, nx, Npackets, link_buffers)
    if link is not None:
        link.seed(ctx)
    U0 = model.max_speed()
    Fr = U0 / Cg
    T = T_Fr / Fr ** 2
    dt = CFL_fraction * dx / U0
    Nsteps = math.ceil(T / dt)
    packet_step_start = math.ceil(packet_delay_steps / dt)
    log(parameter_block(nx, Npackets, near_inertial_factor * f, dt, T, packet_delay_steps, steps_per_save,
                        packet_steps_per_save, f, Cg, U_g, U0, Fr, K_d2, two_layer=True))
    ens = PacketEnsemble(x, k, L, f, Cg, nx, K_d2, shear=shear, k_scale=2 * math.pi / L, nlayers=2,
                         bump=BUMP_QG, ctx=ctx, shard=(rank, world), bounds=bounds) if Npackets > 0 else None
    t = 0.0
    frames = 1
    if ens is not None:
        ens.write_frame(dt * (packet_step_start - 1), out_dir)
    if rank == 0:
        write_field(model.q(), os.path.join(out_dir, "pv"))
        write_field(np.array([[t]]), os.path.join(out_dir, "pv_time"))
    if link is not None and rank == 0:
        link.bind_owner(ctx)
    if link is not None and rank != 0:
        # a receiving rank runs its snapshots on the packet stream: beside its
        # packet launches the transforms run several times slower (they find
        # no free slots), so in series they cost less (bench.py owner legs)
        ctx.qg_set_stream(False)
        ctx.set_packet_streams(1)  # (the snapshot follows the whole previous launch, not beside its second part)
        loop = ReceiverLoop(link, ens, dt, packet_delay_steps, nsub, packet_intervals, integrator)
    else:
        loop = TwoLayerLoop(model, ens, dt, U0, CFL_fraction, packet_delay_steps, nsub, packet_intervals, integrator,
                            log, link=link)
    # (the reference only plots q every steps_per_save steps in this loop; its
    # pv.bin writes are commented out, qg2layersw_raytrace.m:211-239)
    log.start()
    while loop.t <= T and (max_steps is None or loop.steps < max_steps):
        if loop.step() and (loop.steps - packet_step_start + 1) % packet_steps_per_save == 0:
            loop.flush()
            ens.write_frame(loop.t, out_dir)
            frames += 1
        log.progress(loop.steps, Nsteps)
    loop.flush()
    loop.settle()
    if link is not None:
        link.close()
    ctx.synchronize()
    ctx.set_timing(timing)
    log.finish()
    log.close()
    dt, dts, step, t = loop.dt, loop.dts, loop.steps, loop.t
    U0 = getattr(loop, "U0", U0)  # (a receiving rank never sees the owner's U0)
    return dict(dt=dt, dts=dts, Nsteps=Nsteps, steps=step, packet_frames=frames, t=t, U0=U0,
                packet_step_start=packet_step_start)
