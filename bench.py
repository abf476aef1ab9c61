"""Throughput bench: packet-steps/s @ 512^2 field, 1e6 packets; 1/2/4/8 GPUs.

Workload (BASELINE.json configs[3], the metric's config): two-layer QG
background (qg2layersw_raytrace.m: L = 20, wavenumbers scaled by 2*pi/L,
shear_strength 0.5, packets advected in layer 1 so interpolate's y-period is
2*nx), two spectral snapshots (prev_qk, qk) prepared on the GPU by grid_U
(swrt_set_field_qk), 1e6 packets on the omega0 = 4f ring (f = 3, Cg = 1,
Ug = 0.2).  One bench step = one PDE interval dt = 0.25*dx/U0
(CFL_fraction of qg2layersw_raytrace.m:31) advanced by `--substeps` (5)
fused leapfrog steps with the interpolate_U time blend, i.e. packet steps
of 0.05*dx/U0 — the step SURVEY §8d's metric is defined on (qgsw_raytrace.m's
CFL 0.05, :29,70).  A packet-step is the same work at any dt (drift, 36-tap
U + grad U of both snapshots, kick, drift); dt only sets how far packets
move between re-binnings (`--rebin-every` 20 steps here).  Synthetic data:
random phase ring spectrum 10 < |k| <= 30 (initial_q's ring), normalised so
max|U| = Ug; a second snapshot with slightly rotated phases.

Multi-GPU: one process per GPU, packets sharded by rank, field replicated,
no data-path collective; barrier + device sync around the timed region, max
time over ranks.  `--scaling strong` (default): the metric's fixed 1e6-packet
ensemble split over the ranks (configs[3], "1e6 packets, sharded
8xMI355X"); `--scaling weak`: `--packets` per GPU.  `--gpus N` without a
torch.distributed environment launches `python -m torch.distributed.run
--nproc-per-node N bench.py ...` as a CHILD process (never an exec) and
relays its rank-0 line; under torch.distributed.run, WORLD_SIZE must equal
`--gpus`.  At N = 1 the line also carries `strong_scaling_forecast`: the
same workload timed at the shard sizes of 2/4/8 GPUs.

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "packet-steps/sec @ 512² field, 1e6 packets; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E peak (MI355X_MICROARCH.md, chip table)
BYTES_STEADY = 1792          # 32+32 state + 1 snap * 6 fields * 36 taps * 8 B
BYTES_BLEND = 3520           # 32+32 state + 2 snaps * 6 * 36 * 8 B


def ring_spectrum(nx, kmin, kmax_ring, rng, phase_shift=0.0):
    """Half-plane qk with unit-amplitude random phases on kmin < |k| <= kmax_ring."""
    kmax = nx // 2 - 1
    qk = np.zeros((2 * kmax + 1, kmax + 1), dtype=np.complex128)
    ph = rng.uniform(0, 2 * np.pi, qk.shape) + phase_shift
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(0, kmax + 1)[None, :]
    r2 = kx * kx + ky * ky
    mask = (r2 > kmin * kmin) & (r2 <= kmax_ring * kmax_ring)
    qk[mask] = np.exp(1j * ph[mask])
    return qk


def broadband_spectrum(nx, K_d2, ks, rng):
    """SURVEY §8(d)'s broadband variant: psi-hat with random phases and
    |psi-hat| ~ |k|^-3 for 1 <= |k| <= 0.75 kmax (k in grid units), handed to
    grid_U as q-hat = -(K_d2 + K^2) psi-hat (its inversion, grid_U.m:2)."""
    kmax = nx // 2 - 1
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(0, kmax + 1)[None, :]
    r = np.sqrt(kx * kx + ky * ky)
    ph = rng.uniform(0, 2 * np.pi, r.shape)
    mask = (r >= 1) & (r <= 0.75 * kmax)
    psi = np.zeros(r.shape, dtype=np.complex128)
    psi[mask] = r[mask] ** -3.0 * np.exp(1j * ph[mask])
    K2 = (kx * ks) ** 2 + (ky * ks) ** 2
    return -(K_d2 + K2) * psi


def build_workload(ctx, args, lo, hi, n_total):
    """The replicated field (every rank draws the same spectra from `seed`)
    and this rank's packets [lo, hi) of the n_total-packet ensemble (the same
    ensemble at any world size: positions drawn for all n_total packets,
    ring angles 2*pi*i/n_total)."""
    rng = np.random.default_rng(args.seed)
    nx, L, f, Cg, Ug = args.nx, 20.0, 3.0, 1.0, 0.2
    K_d2 = f / Cg
    ks = 2 * np.pi / L
    if getattr(args, "field", "ring") == "broadband":
        qk1 = broadband_spectrum(nx, K_d2, ks, rng)
    else:
        qk1 = ring_spectrum(nx, 10, 30, rng)
    rng2 = np.random.default_rng(args.seed + 1)
    qk2 = qk1 * np.exp(1j * rng2.normal(0, 0.05, qk1.shape))
    # normalise to max|U| = Ug (initial_q, qg2layersw_raytrace.m:279-280)
    ctx.set_field_qk(0, qk1, nx, L, K_d2, 0.0, ks, 2 * nx)
    p = ctx.get_field_grid(0, nx)
    scale = Ug / math.sqrt(float((p[0] ** 2 + p[1] ** 2).max()))
    qk1 *= scale
    qk2 *= scale
    shear = 0.5
    nslots = 1 if args.mode == "steady" else 2
    ctx.set_field_qk(0, qk1, nx, L, K_d2, shear, ks, 2 * nx)
    if nslots == 2:
        ctx.set_field_qk(1, qk2, nx, L, K_d2, shear, ks, 2 * nx)
        set_interval_snapshots(ctx, qk2, rng2, nx, L, K_d2, shear, ks, getattr(args, "intervals", 1))
    p = ctx.get_field_grid(0, nx)
    U0 = math.sqrt(float((p[0] ** 2 + p[1] ** 2).max()))
    dt = 0.25 * (L / nx) / U0  # qg2layersw_raytrace.m:31,78
    w0 = 4.0
    wf = math.sqrt((w0 ** 2 - 1) * f ** 2 / Cg ** 2)
    i = np.arange(lo + 1, hi + 1, dtype=np.float64)
    k = np.stack([wf * np.cos(2 * np.pi * i / n_total), wf * np.sin(2 * np.pi * i / n_total)], axis=1)
    if getattr(args, "positions", "uniform") == "stratified":
        # diagnostic: every 16x16-cell tile gets the same number of packets
        N = hi - lo
        nt = max(1, nx // 16)
        t = np.arange(N) % (nt * nt)
        x = np.stack([(t // nt) * 16 + 16 * rng.random(N), (t % nt) * 16 + 16 * rng.random(N)], axis=1) * (L / nx)
    elif getattr(args, "positions", "uniform") in ("band", "yband"):
        x = (L * rng.random((n_total, 2)) - L / 2)[lo:hi]
        c = 0 if args.positions == "band" else 1
        x[:, c] = (x[:, c] + L / 2) / args.band_parts - L / 2
    else:
        x = (L * rng.random((n_total, 2)) - L / 2)[lo:hi]
    return dict(nx=nx, L=L, f=f, gH=Cg ** 2, dt=dt, nslots=nslots, x=x, k=k, qk1=qk1, qk2=qk2,
                K_d2=K_d2, ks=ks, shear=shear, intervals=getattr(args, "intervals", 1) if nslots == 2 else 1,
                seed=args.seed)


def set_interval_snapshots(ctx, qk2, rng2, nx, L, K_d2, shear, ks, intervals):
    """Slots 2..intervals: the later snapshots of `intervals` consecutive PDE
    intervals (--intervals), each a further small phase rotation of the
    previous one (rng2 continues the stream that made qk2)."""
    qk = qk2
    for s in range(2, intervals + 1):
        qk = qk * np.exp(1j * rng2.normal(0, 0.05, qk.shape))
        ctx.set_field_qk(s, qk, nx, L, K_d2, shear, ks, 2 * nx)


def with_intervals(ctx, w, K):
    """The workload `w` advanced K PDE intervals per call (one
    swrt_advance_intervals call, 5K steps per launch): slots 2..K get the
    snapshots build_workload makes for --intervals K (the same seed stream)."""
    if w["nslots"] != 2 or K <= w["intervals"]:
        return dict(w, intervals=K if w["nslots"] == 2 else 1)
    rng2 = np.random.default_rng(w["seed"] + 1)
    rng2.normal(0, 0.05, w["qk1"].shape)  # the draw that made qk2
    set_interval_snapshots(ctx, w["qk2"], rng2, w["nx"], w["L"], w["K_d2"], w["shear"], w["ks"], K)
    return dict(w, intervals=K)


def step(ctx, w, sub):
    """One bench step: `intervals` PDE intervals of `sub` leapfrog steps
    (interval i blends snapshots i, i+1; one call, swrt_advance_intervals)."""
    h = w["dt"] / sub
    if w.get("intervals", 1) > 1:
        ctx.advance_intervals([h] * w["intervals"], sub, w["f"], w["gH"], alpha0=0.5 / sub, dalpha=1.0 / sub,
                              bump=sw.BUMP_QG)
        return
    ctx.advance(h, sub, w["f"], w["gH"], nslots=w["nslots"], alpha0=0.5 / sub, dalpha=1.0 / sub,
                bump=sw.BUMP_QG)


def host_cpu():
    """Where the CPU baseline ran: nproc, the process's CPU affinity, the
    cgroup CPU quota (cores) when one is set, and the CPU model."""
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = None
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "cgroup_cpu_quota": quota, "cpu_model": model}


def cpu_baseline(ctx, w, target_s, threads):
    """The C oracle's CPU-arranged leapfrog (oracle_leapfrog_fast: the same
    bits as the restatement, interleaved nodes, weights shared by both
    snapshots) built here with -O3 -march=native, OpenMP over packets, timed
    on the same fields on a bounded sample."""
    import tempfile

    from oracle import cbind
    nx = w["nx"]
    p0 = ctx.get_field_grid(0, nx)
    p1 = ctx.get_field_grid(1, nx) if w["nslots"] == 2 else None
    L, flags = cbind.cpu_lib(tempfile.mkdtemp(prefix="swrt_cpu_"))
    default_threads = L.oracle_num_threads()
    L.oracle_set_threads(threads)
    nthreads = L.oracle_num_threads()

    def run(n, steps):
        t0 = time.perf_counter()
        cbind.leapfrog_fast(p0, p1, 0.5, 0.0, nx, 2 * nx, w["L"] / nx, sw.BUMP_QG, w["x"][:n], w["k"][:n],
                            w["dt"] / 5, steps, w["f"], w["gH"], L=L)
        return time.perf_counter() - t0

    n = min(8192 * max(1, nthreads // 4), w["x"].shape[0])
    run(n, 1)  # warm-up: OpenMP thread start, page faults
    t = run(n, 4)
    s1 = max(4, int(1.0 * 4 / max(t, 1e-9)))  # ~1 s calibration run
    t = run(n, s1)
    steps = max(1, int(target_s * s1 / max(t, 1e-9)))
    t = run(n, steps)
    L.oracle_set_threads(default_threads)
    return {"value": n * steps / t, "unit": "packet-steps/s", "cores": int(nthreads), "kind": "port",
            "sample": f"{n} packets x {steps} leapfrog steps (dt 0.05*dx/U0) of the bench's {nx}^2 two-snapshot "
                      f"field, oracle_leapfrog_fast (oracle/swrt_oracle.c, same bits as the restatement), "
                      f"{nthreads} OpenMP threads, {t:.1f} s",
            "build": flags, "host": host_cpu()}


def driver_step(ctx, w, args, dev, distributed, n_total, integrator="leapfrog", nsteps=None):
    """The end-to-end qg2layersw_raytrace step on this GPU (swraytracing_amd.qg.
    TwoLayerLoop, the driver's own loop body): CFL rule, 2-layer PDE step, U0
    read-back, grid_U snapshot of the new qk and the packet interval of all
    this rank's packets (`--substeps` leapfrog substeps, or the reference's
    own ode23 over the interval), the PDE on its own stream beside the
    packets.  Outside the metric's timed region; reported as extra keys so
    the driver-level rates are observed by the same run."""
    nx, L, f, Cg = w["nx"], w["L"], w["f"], math.sqrt(w["gH"])
    nsteps = args.driver_steps if nsteps is None else nsteps
    w_in = w
    qk = np.stack([w["qk1"], -w["qk1"]], axis=2)  # the driver's (q1, -q1) layers
    owner_form = distributed and args.driver_pde == "owner" and integrator == "leapfrog"
    if owner_form:
        # the PDE-owner form across the ranks (qg.py OwnerLink / ReceiverLoop):
        # the ensemble re-split by dist.owner_bounds (every rank draws all
        # n_total packets from the same seed: build_workload), rank 0 steps the
        # PDE and broadcasts each step's top-layer qk and dt
        from swraytracing_amd.dist import OwnerLink, owner_bounds
        full = build_workload(ctx, args, 0, n_total, n_total)
        lo, hi = owner_bounds(n_total, args.world, args.owner_weight)[args.rank]
        w = dict(w, x=full["x"][lo:hi], k=full["k"][lo:hi])
        link = OwnerLink(nx, args.dist_backend)
    model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
    ens = sw.PacketEnsemble(w["x"], w["k"], L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * math.pi / L, nlayers=2,
                            bump=sw.BUMP_QG, ctx=ctx)
    U0 = model.max_speed()
    if owner_form and args.rank != 0:
        ctx.qg_set_stream(False)
        ctx.set_packet_streams(1)
        link.seed(ctx)
        loop = sw.ReceiverLoop(link, ens, 0.25 * (L / nx) / U0, 0.0, nsub=args.substeps)
    else:
        if owner_form:
            link.bind_owner(ctx)
            link.seed(ctx)
        loop = sw.TwoLayerLoop(model, ens, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=args.substeps,
                               integrator=integrator, speculate=bool(args.speculate),
                               link=link if owner_form else None)
    # AB1/AB2 start-up and first-use allocations: the snapshot renaming (qg.py
    # TwoLayerLoop) allocates its spare slot buffers during the first steps, a
    # hipMalloc each — outside the timed steps.  Then warm-up steps until
    # DRIVER_WARM_S of driver work have run: this phase follows seconds of
    # host-only work (the CPU baseline) in the default run, and a GPU coming
    # back from idle holds a different clock for its first milliseconds
    # (0.297-0.304 vs 0.277-0.280 ms per step at 1e6 with and without the
    # idle gap before a 16-step warm-up, profiles/r05_qg_copy)
    for _ in range(args.driver_warmup):
        loop.step()
    if owner_form:  # every rank takes the same steps (each is a collective)
        for _ in range(OWNER_WARM_STEPS):
            loop.step()
    else:
        tw = time.perf_counter()
        while time.perf_counter() - tw < args.driver_warm_s:
            loop.step()
    loop.flush()
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    if distributed:
        dist.barrier()
    nd0 = len(loop.dts)
    chained0 = ctx.debug_get(sw._lib.DEBUG_ODE23_CHAINED)
    ctx.clock_stamp(0)
    t0 = time.perf_counter()
    for _ in range(nsteps):
        loop.step()
    loop.flush()
    ctx.clock_stamp(1)
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    try:
        clk = ctx.clock_ghz()[0]
    except sw.SwrtError:  # no CU ran both probe waves (see timed)
        clk = None
    if distributed:
        el = max_over_ranks(el, backend=args.dist_backend)
    ms = el / nsteps * 1e3
    what = (f"TwoLayerLoop.step: CFL rule + 2-layer PDE step + U0 read-back + grid_U snapshot + "
            + (f"{args.substeps} leapfrog substeps" if integrator == "leapfrog" else "ode23 over the interval "
               "(qg2layersw_raytrace.m:195: RelTol 1e-3, AbsTol 1e-6, MaxStep 0.1*dt)")
            + f" of {w['x'].shape[0]} packets/GPU (qg2layersw_raytrace.m:152-197)")
    timed_dts = loop.dts[nd0:]
    out = {"ms_per_pde_step": ms, "steps": nsteps, "what": what, "clock_ghz_observed": clk,
           # the CFL rule (qg2layersw_raytrace.m:156-165) re-forms the exponential propagators when dt changes
           "dt_changes": int(sum(1 for a, b in zip(loop.dts[nd0 - 1:], timed_dts) if a != b))}
    if owner_form:
        loop.settle()
        out["pde"] = f"owner form (rank 0 steps the PDE, owner weight {args.owner_weight})"
        ctx.qg_set_stream(bool(args.qg_stream))
        ctx.set_packet_streams(args.packet_streams)
        ctx.packets_set(w_in["x"], w_in["k"])
    if integrator == "leapfrog":
        out["packet_steps_per_s"] = n_total * args.substeps / (ms / 1e3)
    else:
        out["packet_intervals_per_s"] = n_total / (ms / 1e3)
        # the controller's own counts over warm-up and timed intervals (attempts include rejected ones)
        st = loop.group.ode23_stats
        if st["intervals"]:
            out["ode23_per_interval"] = {k: st[k] / st["intervals"] for k in ("steps", "failed", "attempts")}
        # timed intervals whose stage 1 the previous one queued (swrt_ode23_chain_next)
        out["ode23_chained_intervals"] = ctx.debug_get(sw._lib.DEBUG_ODE23_CHAINED) - chained0
    return out


def pde_alone(ctx, w, args, dev, nsteps=None):
    """The driver loop without packets (TwoLayerLoop with no ensemble): CFL
    rule, 2-layer PDE step and the U0 read-back (qg2layersw_raytrace.m:152-181),
    i.e. the replicated part of every rank's driver step."""
    nx, L, f, Cg = w["nx"], w["L"], w["f"], math.sqrt(w["gH"])
    nsteps = nsteps or args.driver_steps
    qk = np.stack([w["qk1"], -w["qk1"]], axis=2)
    model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
    U0 = model.max_speed()
    loop = sw.TwoLayerLoop(model, None, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=args.substeps,
                           speculate=bool(args.speculate))
    for _ in range(args.driver_warmup):
        loop.step()
    tw = time.perf_counter()
    while time.perf_counter() - tw < args.driver_warm_s:  # (as in driver_step)
        loop.step()
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(nsteps):
        loop.step()
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / nsteps * 1e3


def driver_forecast(ctx, w, args, dev, n_total, full):
    """End-to-end strong-scaling forecast of the 2-layer driver: `driver_step`
    timed on one GPU with rank 0's shard of a G-GPU run (the first
    ceil(n_total/G) packets) beside the full replicated PDE, G = 2, 4, 8;
    efficiency = rate(shard) / rate(all n_total on one GPU).  With the PDE
    alone and the packets alone (strong_scaling_forecast) beside it, `bound`
    names the term that sets the step: the PDE when its own step time exceeds
    the packets'."""
    pde_ms = pde_alone(ctx, w, args, dev, nsteps=args.forecast_driver_steps)
    out = {"pde_alone_ms": pde_ms,
           "what": "TwoLayerLoop.step with 1e6/G packets on one GPU (full replicated 2-layer PDE + snapshot + "
                   f"{args.substeps} leapfrog substeps); pde_alone_ms: the same loop without packets"}
    rate_full = full["packet_steps_per_s"]
    for G in (2, 4, 8):
        n = -(-n_total // G)
        ws = dict(w, x=w["x"][:n], k=w["k"][:n])
        d = driver_step(ctx, ws, args, dev, False, n, nsteps=args.forecast_driver_steps)
        r = {"packets_per_gpu": n, "ms_per_pde_step": d["ms_per_pde_step"],
             "value_1gpu": d["packet_steps_per_s"], "forecast_value": G * d["packet_steps_per_s"],
             "efficiency": d["packet_steps_per_s"] / rate_full}
        out[str(G)] = r
    return out


def _time_loop(ctx, loop, args, dev, nsteps):
    """ms per step of a driver loop on this GPU: start-up steps, then steps
    for DRIVER_WARM_S seconds (see driver_step), then `nsteps` timed."""
    for _ in range(args.driver_warmup):
        loop.step()
    tw = time.perf_counter()
    while time.perf_counter() - tw < args.driver_warm_s:
        loop.step()
    loop.flush()
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(nsteps):
        loop.step()
    loop.flush()
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    return (time.perf_counter() - t0) / nsteps * 1e3


def _owner_links():
    """The OwnerLink of both legs on one GPU: every step's export (owner) or
    dt read and snapshot (receiver) on the link's own stream with its event
    ordering — only the broadcast itself is left out (its buffer already
    holds what it would carry)."""
    from swraytracing_amd.dist import OwnerLink

    class OneGPU(OwnerLink):  # the link's stream, export and snapshot, without the broadcasts
        def __init__(self, nx, dt=0.0, nbuf=5):
            super().__init__(nx, "nccl", nbuf=nbuf)
            self.fixed_dt = dt

        def _bcast(self, b, async_op=False):
            return None

        def _send_dt(self, dt):
            pass

        def _recv_dt(self, b):
            return self.fixed_dt

    return OneGPU


OWNER_WEIGHTS = (0.0, 0.05, 0.1, 0.25, 0.5, 1.0)


def owner_forecast(ctx, w, args, dev, n_total, full_ms):
    """The PDE-owner form of the sharded 2-layer driver (qg.py: rank 0 steps
    the PDE, publishes each step's top-layer qk and dt; every other rank only
    builds its snapshot from it and advances its packets), forecast from its
    two legs measured on this one GPU, each timed as the loop the rank runs:
      owner leg:    TwoLayerLoop with n0 packets + the export of qk (PDE, CFL
                    read-back, snapshot, packets; the broadcast itself omitted)
      receiver leg: ReceiverLoop with nr packets (swrt_snapshot_qk from a
                    device buffer on the QG stream + the packet interval)
    with n0 = N w/(w + G - 1) and nr = N/(w + G - 1) (dist.owner_bounds) for
    owner weights w in OWNER_WEIGHTS; per G the step is max(owner, receiver)
    at the best w, efficiency = the one-GPU driver step (all N) / (G x step)."""
    OneGPU = _owner_links()
    nx, L, f, Cg = w["nx"], w["L"], w["f"], math.sqrt(w["gH"])
    qk = np.stack([w["qk1"], -w["qk1"]], axis=2)
    nsteps = args.forecast_driver_steps
    legs = {}

    def ensemble(n):
        return sw.PacketEnsemble(w["x"][:n], w["k"][:n], L, f, Cg, nx, f / Cg, shear=0.5, k_scale=2 * math.pi / L,
                                 nlayers=2, bump=sw.BUMP_QG, ctx=ctx)

    def owner_ms(n0):
        if ("o", n0) not in legs:
            model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)
            U0 = model.max_speed()
            ens = ensemble(n0)  # (n0 = 0: an empty ensemble — the context then holds no packets, as the owner's)
            loop = sw.TwoLayerLoop(model, ens, 0.25 * (L / nx) / U0, U0, 0.25, 0.0, nsub=args.substeps,
                                   speculate=bool(args.speculate), link=OneGPU(nx).bind_owner(ctx))
            legs[("o", n0)] = _time_loop(ctx, loop, args, dev, nsteps)
            loop.settle()
        return legs[("o", n0)]

    def receiver_ms(nr):
        if ("r", nr) not in legs:
            ctx.qg_set_stream(False)  # a receiving rank's snapshots run in series with its packets (qg.py)
            ctx.set_packet_streams(1)
            model = sw.QGModel.two_layer(qk, nx, f, Cg, L=L, ctx=ctx)  # (a receiving rank holds one too)
            dt = 0.25 * (L / nx) / model.max_speed()
            link = OneGPU(nx, dt)
            for b in link.bufs:  # every step 'receives' this qk and dt
                link._export(ctx, b, dt)
            loop = sw.ReceiverLoop(link, ensemble(nr), dt, 0.0, nsub=args.substeps)
            legs[("r", nr)] = _time_loop(ctx, loop, args, dev, nsteps)
            ctx.qg_set_stream(bool(args.qg_stream))
            ctx.set_packet_streams(args.packet_streams)
        return legs[("r", nr)]

    out = {"what": "PDE-owner form (qg.py OwnerLink/ReceiverLoop): rank 0 = TwoLayerLoop with n0 packets + qk export; "
                   "ranks 1..G-1 = ReceiverLoop with nr packets (snapshot from the broadcast qk + packets); both "
                   "legs timed on this GPU; step = max(owner, receiver) at the best owner weight",
           "assumption": "the per-step RCCL broadcast of the top-layer qk (2.1 MB at 512^2) + dt from rank 0 is not "
                         "measured (one GPU here): it is queued behind the owner's export and ahead of the "
                         "receivers' snapshot, and is assumed to complete while their previous packet interval runs",
           "one_gpu_ms": full_ms, "weights": list(OWNER_WEIGHTS)}
    for G in (2, 4, 8):
        from swraytracing_amd.dist import owner_bounds
        tried = []
        for wt in OWNER_WEIGHTS:
            b = owner_bounds(n_total, G, wt)
            n0, nr = b[0][1] - b[0][0], b[1][1] - b[1][0]
            o, r = owner_ms(n0), receiver_ms(nr)
            tried.append({"owner_weight": wt, "packets_owner": n0, "packets_per_receiver": nr, "owner_ms": o,
                          "receiver_ms": r, "step_ms": max(o, r)})
        best = min(tried, key=lambda d: d["step_ms"])
        out[str(G)] = dict(best, forecast_value=n_total * args.substeps / (best["step_ms"] / 1e3),
                           efficiency=full_ms / (G * best["step_ms"]), legs=tried)
    return out


DRIVER_WARM_S = 0.3  # seconds of untimed driver steps before each driver-step measurement
OWNER_WARM_STEPS = 100  # ... in the owner form, a step count (every step is a collective)
FP64_LANE_OPS_PEAK = 256 * 4 * 16 * 2.4e9  # fp64 VALU lane-ops/s (78.6 TFLOP/s spec counts an FMA as 2)
LDS_CYCLES_PEAK = 256 * 2.4e9               # LDS-array cycles/s over the chip (one array per CU, 2.4 GHz)
# fp64 operations one packet-step of the reference arithmetic needs (each +, -, *, /, sqrt, floor one op;
# the six Lagrange weights per direction and the 36 products wx_i*wy_j computed once per step and shared
# by every field, as any implementation may; v_y = -u_x on streamfunction fields):
#   cell + fractional offset (interpolate.m:21-30): x/dx, mod (div, floor, mul, sub), 1 + floor,
#     1 + xl - i0; 2 directions x 9                                            18
#   Lagrange weights (:32-40): 6 factors (a - j + bump) x 2 ops + 30 mul + 30 div, x 2 directions  144
#   tap products wx_i*wy_j (:45-48)                                           36
#   10 stencil sums (5 fields x 2 snapshots) x (36 mul + 35 add)             710
#   blend (interpolate_U.m:19-23): (1 - alpha) + 5 fields x (2 mul, add)      16
#   leapfrog (ode_symplectic.m:10-21): omega (k*k, l*l, add, gH*, f^2 +, sqrt) 6, gH*k/omega and
#     gH*l/omega 4, half-step scaling 2, two drifts applied 4; kick: x 2 x (mul, add),
#     k 2 x (3 mul, add, sub)                                                  30
ALG_OPS_PER_PACKET_STEP = 18 + 144 + 36 + 710 + 16 + 30  # = 954 (two-snapshot blend)
ALG_OPS_STEADY = 18 + 144 + 36 + 5 * 71 + 30             # = 583 (one snapshot)


def load_pmc(config_key):
    """PMC record of this bench configuration (tools/pmc_collect.sh ->
    profiles/pmc.json), only if it was collected on the device code being
    timed (its code_object_sha256 = the loaded libswrt's .hip_fatbin hash);
    returns (record or None, note)."""
    path = os.path.join(ROOT, "profiles", "pmc.json")
    try:
        rec = json.load(open(path)).get(config_key)
    except (OSError, ValueError):
        rec = None
    if rec is None:
        return None, f"no PMC record for {config_key} in profiles/pmc.json (tools/pmc_collect.sh)"
    have = sw._lib.device_code_sha256()
    if rec.get("code_object_sha256") != have:
        return None, (f"profiles/pmc.json[{config_key}] was collected on device code "
                      f"{str(rec.get('code_object_sha256'))[:12]}, the library timed is {have[:12]}: frac not computed")
    return rec, "PMC bound to device code " + have[:12]


def roofline(pmc, N, nx, nslots, steps_per_launch, avg_launch_s, launches, timing_every):
    """The dominant kernel (tile_leapfrog_kernel) against the resource that
    bounds it.  The bit-exact stencil (mul then add, no FMA) is
    fp64-VALU-issue bound: achieved = the kernel's PMC-counted VALU
    instructions per launch x 64 lanes / its live HIP-event launch time,
    peak = 256 CUs x 4 SIMDs x 16 fp64 lanes x 2.4 GHz.  HBM and the LDS
    array are reported beside it as fractions of their own peaks."""
    ps = N * steps_per_launch
    B = BYTES_BLEND if nslots == 2 else BYTES_STEADY
    ops = ALG_OPS_PER_PACKET_STEP if nslots == 2 else ALG_OPS_STEADY
    r = {"bound": "valu-fp64-issue", "achieved": None, "peak": FP64_LANE_OPS_PEAK / 1e12, "unit": "Tlane-op/s",
         "frac": None, "traffic": None,
         "avg_launch_ms": avg_launch_s * 1e3, "timed_launches": launches, "timing_every": timing_every,
         "packet_steps_per_launch": ps,
         # the reference arithmetic's own fp64 operations (ALG_OPS_PER_PACKET_STEP) over the same time and
         # peak: instruction overhead (index math, exact-division sequences, loads' address arithmetic)
         # does not count here, so this fraction cannot be raised by issuing more instructions
         "algorithmic_ops_per_packet_step": ops,
         "algorithmic_frac": ops * ps / avg_launch_s / FP64_LANE_OPS_PEAK,
         # SURVEY §8d's algorithmic bytes (taps counted as if each were read from HBM; they are
         # re-read from LDS): an effective gather bandwidth, not an HBM fraction
         "effective_gather_gbs": ps * B / avg_launch_s / 1e9, "gather_bytes_per_packet_step": B}
    if pmc is None:
        return r
    valu = pmc["SQ_INSTS_VALU"]
    ach = valu * 64.0 / avg_launch_s
    traffic = (2.0 * pmc["FETCH_SIZE"] + pmc["WRITE_SIZE"]) * 1024.0  # KiB; FETCH doubled (gfx950)
    compulsory = N * (36 + 36) + nslots * (nx + 5) ** 2 * 48  # state+perm in/out, the snapshots once
    hbm = traffic / avg_launch_s / 1e9
    pmc_s = pmc["pmc_kernel_ns"] * 1e-9
    r.update({
        "achieved": ach / 1e12, "frac": ach / FP64_LANE_OPS_PEAK,
        "valu_instructions_per_launch": valu,
        "valu_per_wave_step": valu / (N / 64.0 * steps_per_launch),
        "traffic": traffic, "hbm_gbs": hbm, "hbm_frac": hbm / HBM_PEAK_GBS,
        "compulsory_bytes_per_launch": compulsory, "traffic_over_compulsory": traffic / compulsory,
        "lds_frac": pmc["SQ_LDS_IDX_ACTIVE"] / (LDS_CYCLES_PEAK * pmc_s),
        "lds_conflict_factor": pmc["SQ_LDS_IDX_ACTIVE"] / max(1.0, pmc["SQ_LDS_IDX_ACTIVE"] - pmc["SQ_LDS_BANK_CONFLICT"]),
        "wait_frac": pmc["SQ_WAIT_ANY"] / max(1.0, pmc["SQ_WAVE_CYCLES"]),
        "pmc_kernel_ms": pmc_s * 1e3,
        "source": "profiles/pmc.json: " + pmc.get("source", "") + "; kernel " + pmc.get("kernel", "")})
    if pmc.get("GRBM_GUI_ACTIVE"):
        # GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs: the engine clock the
        # kernel actually ran at (below the 2.4 GHz the peaks assume under this load)
        clk = pmc["GRBM_GUI_ACTIVE"] / 8.0 / pmc_s
        r.update({"clock_ghz_measured": clk / 1e9,
                  "frac_at_measured_clock": ach / (FP64_LANE_OPS_PEAK * clk / 2.4e9),
                  "algorithmic_frac_at_measured_clock": r["algorithmic_frac"] * 2.4e9 / clk,
                  "lds_frac_at_measured_clock": pmc["SQ_LDS_IDX_ACTIVE"] / (256 * clk * pmc_s)})
    return r


def add_observed_clock(r, ghz, spread):
    """The clock the timed region actually ran at (swrt_clock_stamp probes,
    rank 0's GPU) and the fractions re-based to it: peak x ghz / 2.4 (the
    chip lowers its clock under load, and boxes differ — this is what makes
    a throughput change attributable to code rather than to the box)."""
    r["clock_ghz_observed"] = ghz
    r["clock_probe_spread"] = spread
    r["clock_note"] = ("median over CUs of s_memtime cycles / s_memrealtime seconds between the CU's first start "
                       "and last end probe wave around the timed region (same-CU pairs: the cycle counters of "
                       "different CUs are not aligned); *_at_observed_clock = the fraction against the peak at "
                       "that clock; null when no CU ran both a start and an end probe (a GPU shared by ranks)")
    if ghz and ghz > 0:
        s = 2.4 / ghz
        if r.get("frac") is not None:
            r["frac_at_observed_clock"] = r["frac"] * s
        r["algorithmic_frac_at_observed_clock"] = r["algorithmic_frac"] * s
    return r


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (ranks); without a torch.distributed environment N > 1 launches the ranks as a child "
                         "torch.distributed.run; under one it must equal WORLD_SIZE (default: WORLD_SIZE)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong",
                    help="strong: --packets in total, sharded over the ranks (the metric's fixed 1e6); "
                         "weak: --packets per GPU")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--nx", type=int, default=512)
    ap.add_argument("--packets", type=int, default=1_000_000,
                    help="packets in total (strong scaling) or per GPU (weak)")
    ap.add_argument("--substeps", type=int, default=5,
                    help="leapfrog steps per bench step (PDE interval 0.25*dx/U0; 5 -> 0.05*dx/U0 per step)")
    ap.add_argument("--intervals", type=int, default=1,
                    help="PDE intervals per bench step, one call (swrt_advance_intervals; up to 4 per launch)")
    ap.add_argument("--mode", choices=["blend", "steady"], default="blend")
    ap.add_argument("--seed", type=int, default=146)
    ap.add_argument("--positions", choices=["uniform", "stratified", "band", "yband"], default="uniform",
                    help="initial packet positions (stratified: equal packets per tile; band: all packets in the "
                         "first 1/--band-parts of the domain in x, a spatial-shard diagnostic)")
    ap.add_argument("--band-parts", type=int, default=8)
    ap.add_argument("--field", choices=["ring", "broadband"], default="ring",
                    help="flow: the drivers' ring spectrum 10 < |k| <= 30 (initial_q), or SURVEY 8(d)'s broadband "
                         "|psi| ~ |k|^-3 up to 0.75 kmax (every scale, every tile)")
    ap.add_argument("--gather-mode", type=int, default=0, choices=[0, 1],
                    help="headline stencil arithmetic: 0 bit-exact (default), 1 FMA (tolerance; PMC diagnostics)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fma", action="store_true",
                    help="skip the extra line of the opt-in FMA gather mode (swrt_set_gather_mode 1, tolerance parity)")
    ap.add_argument("--no-forecast", action="store_true",
                    help="at N = 1, skip the strong-scaling forecast (the workload at 2/4/8-GPU shard sizes)")
    ap.add_argument("--forecast-intervals", type=int, default=4,
                    help="at N = 1, also forecast with this many PDE intervals per call (1: skip)")
    ap.add_argument("--rebin-every", type=int, default=20, help="steps between spatial re-binning (0: off)")
    ap.add_argument("--tile", type=int, default=0, help="binning tile (cells); 0: automatic")
    ap.add_argument("--kernel", type=int, default=0, help="0 auto, 1 per-packet, 2 LDS tile")
    ap.add_argument("--sparse-tiles", type=int, default=0, choices=[0, 1, 2],
                    help="LDS-tiled launches: sparse-tile shape (256 threads, reads 3 taps ahead) 0 auto, 1 never, "
                         "2 always (same bits)")
    ap.add_argument("--packet-streams", type=int, default=2, choices=[1, 2],
                    help="LDS-tiled launches split over 1 or 2 streams (swrt_set_packet_streams; same bits; "
                         "2 is the library default)")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend (nccl = RCCL over xGMI); gloo lets ranks share a GPU")
    ap.add_argument("--timing-every", type=int, default=5,
                    help="HIP-event-time every k-th packet-kernel launch (sampled, inside the timed region)")
    ap.add_argument("--driver-steps", type=int, default=50,
                    help="after the metric, time this many end-to-end driver steps (PDE + snapshot + packets; 0: skip)")
    ap.add_argument("--qg-jfuse", type=int, default=1, choices=[0, 1],
                    help="2-layer PDE: inverse column pass fused with the Jacobian (SWRT_DEBUG_QG_JFUSE; same bits)")
    ap.add_argument("--qg-update-cols", type=int, default=1, choices=[0, 1],
                    help="PDE: J's last forward pass fused into the AB3 update (SWRT_DEBUG_QG_UPDATE_COLS; same bits)")
    ap.add_argument("--qg-stream", type=int, default=1, choices=[0, 1],
                    help="driver steps: the PDE on its own stream beside the packets (1) or on the packet stream (0)")
    ap.add_argument("--speculate", type=int, default=1, choices=[0, 1],
                    help="driver steps: queue the next PDE step before reading U0 (TwoLayerLoop speculate)")
    ap.add_argument("--forecast-driver-steps", type=int, default=100,
                    help="timed driver steps per shard size in driver_step_forecast")
    ap.add_argument("--driver-warm-s", type=float, default=DRIVER_WARM_S,
                    help="then driver steps for this many seconds, untimed (a GPU back from idle; 0: none)")
    ap.add_argument("--driver-warmup", type=int, default=16,
                    help="untimed driver steps before the timed ones (start-up, spare snapshot buffers)")
    ap.add_argument("--driver-pde", choices=["replicated", "owner"], default="replicated",
                    help="N > 1 driver step: every rank steps the PDE (replicated), or rank 0 steps it and broadcasts "
                         "the top-layer qk + dt (owner form, qg.py OwnerLink; its N = 1 forecast is "
                         "driver_step_forecast.owner)")
    ap.add_argument("--owner-weight", type=float, default=0.0,
                    help="owner form: rank 0's packets per packet of another rank (dist.owner_bounds)")
    ap.add_argument("--ode23-steps", type=int, default=16,
                    help="then this many driver steps with the reference's ode23 packet integrator (0: skip)")
    ap.add_argument("--gather", action="store_true",
                    help="after timing, gather all trajectories to rank 0 (one all_gather)")
    return ap.parse_args(argv)


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launcher_cmd(args, argv, env):
    """The child command that runs this bench on `--gpus` ranks, or None when
    this process is itself a rank (WORLD_SIZE set) or one GPU was asked for.
    Raises if a torch.distributed environment disagrees with --gpus."""
    world = env.get("WORLD_SIZE")
    if world is not None:
        if args.gpus is not None and args.gpus != int(world):
            raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
        return None
    if args.gpus is None or args.gpus <= 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)


def relay(cmd):
    """Run the ranks as a child process; the rank-0 JSON line goes to stdout,
    everything else to stderr as it arrives.  Returns the child's exit code."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, env=env)
    for line in proc.stdout:
        t = line.strip()
        if t.startswith("{") and '"metric"' in t:
            print(t, flush=True)
        else:
            print(line, end="", file=sys.stderr, flush=True)
    return proc.wait()


def progress(msg):
    """One line per bench phase on stderr (a run that prints nothing for
    minutes looks hung to the GPU box's watchdog)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _imports():
    """torch and the library, imported only in a rank (never in the launcher)."""
    global torch, dist, sw, gather_packets, max_over_ranks, shard_range
    import torch  # noqa: F401  (first: libswrt binds to the HIP runtime torch loads)
    import torch.distributed as dist  # noqa: F401

    import swraytracing_amd as sw  # noqa: F401
    from swraytracing_amd.dist import gather_packets, max_over_ranks, shard_range  # noqa: F401


def steps_per_launch_of(args, ivs):
    """Packet-steps per launch: a call's substeps run as launches of at most
    `rebin_every` steps, cut at the re-binning points (swrt_advance)."""
    if ivs > 1 and args.rebin_every > 0 and args.rebin_every % args.substeps == 0 and args.kernel in (0, 2):
        return args.substeps * min(ivs, 4, args.rebin_every // args.substeps)  # whole intervals, up to 4
    if args.rebin_every <= 0 or args.rebin_every % args.substeps == 0:
        return min(args.substeps, 64)
    if args.substeps % args.rebin_every == 0:
        return args.rebin_every
    return min(args.substeps, args.rebin_every)  # approximate (uneven chunks)


def timed(ctx, w, args, dev, steps, warmup, barrier=None):
    """warmup untimed steps, then `steps` timed ones bracketed by a device
    sync (and the caller's barrier); returns (elapsed s, sampled kernel ms,
    launches, observed shader clock: (GHz, spread) from swrt_clock_stamp's
    one-wave probes enqueued on the packet stream before the first and after
    the last timed launch)."""
    for _ in range(warmup):
        step(ctx, w, args.substeps)
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    if barrier:
        barrier()
    ctx.set_timing(args.timing_every)
    ctx.kernel_time(reset=True)
    ctx.clock_stamp(0)
    t0 = time.perf_counter()
    for _ in range(steps):
        step(ctx, w, args.substeps)
    ctx.clock_stamp(1)
    ctx.synchronize()
    torch.cuda.synchronize(dev)
    t1 = time.perf_counter()
    if barrier:
        barrier()
    kms, launches = ctx.kernel_time(reset=True)
    ctx.set_timing(0)
    try:
        clk = ctx.clock_ghz()
    except sw.SwrtError:
        # no CU ran both a start and an end probe wave: another process's
        # kernels held the CUs (ranks sharing one GPU); the clock is unobserved
        clk = (None, None)
    return t1 - t0, kms, launches, clk


def strong_scaling_forecast(ctx, w, args, dev, n_total, rate_1gpu, sizes=(2, 4, 8), steps=None):
    """One GPU timed on the packets rank 0 of a G-GPU strong-scaling run
    holds (the first ceil(n_total/G) of the same ensemble) for G = 2, 4, 8:
    forecast value = G x that rate (the field is replicated and the timed path
    has no collective), efficiency = rate(shard) / rate_1gpu (the rate of all
    n_total packets on one GPU; G = 1 in `sizes` times that too)."""
    out = {}
    x, k = w["x"], w["k"]
    steps = steps or args.steps
    for G in sizes:
        n = -(-n_total // G)
        ctx.packets_set(x[:n], k[:n])
        el, kms, launches, (clk, _) = timed(ctx, w, args, dev, steps, args.warmup)
        rate = n * args.substeps * w["intervals"] * steps / el
        out[str(G)] = {"packets_per_gpu": n, "value_1gpu": rate, "forecast_value": G * rate,
                       "efficiency": rate / rate_1gpu if rate_1gpu else None, "ms_per_step": el / steps * 1e3,
                       "avg_launch_ms": (kms / launches) if launches else None, "clock_ghz_observed": clk}
    ctx.packets_set(x, k)
    return out


def intervals_forecast(ctx, w, args, dev, n_total, rate_1gpu, K):
    """The strong-scaling forecast with K PDE intervals per call (swrt_advance_
    intervals, 5K steps per tile launch: the window staging, in-tile sort and
    launch tail paid once per K intervals; each interval blends its own pair of
    K + 1 distinct snapshots, as a driver running the PDE K steps ahead or
    trace_stored does).  Efficiencies against the metric's one-interval 1e6
    rate (`efficiency`) and against this form's own 1e6 rate."""
    wk = with_intervals(ctx, w, K)
    steps = max(1, args.steps // K)  # the same packet-steps per timed region
    out = strong_scaling_forecast(ctx, wk, args, dev, n_total, rate_1gpu, sizes=(1, 2, 4, 8), steps=steps)
    own = out["1"]["value_1gpu"]
    for G, r in out.items():
        r["efficiency_vs_own_1gpu"] = r["value_1gpu"] / own
    out["intervals_per_call"] = K
    out["steps_per_launch"] = args.substeps * min(K, 4)
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    cmd = launcher_cmd(args, argv, os.environ)
    if cmd is not None:
        sys.exit(relay(cmd))
    _imports()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    args.world, args.rank = world, rank
    distributed = world > 1
    ndev = max(1, torch.cuda.device_count())
    device = local % ndev
    torch.cuda.set_device(device)
    if distributed:
        dist.init_process_group(backend=args.dist_backend, init_method="env://")
    dev = torch.device("cuda", device)

    n_total = args.packets if args.scaling == "strong" else args.packets * world
    lo, hi = shard_range(n_total, world, rank)
    ctx = sw.Context(device)
    ctx.set_locality(args.rebin_every, args.tile)
    ctx.set_kernel(args.kernel)
    ctx.set_sparse_tiles(args.sparse_tiles)
    ctx.debug_set(sw._lib.DEBUG_QG_JFUSE, args.qg_jfuse)
    ctx.debug_set(sw._lib.DEBUG_QG_UPDATE_COLS, args.qg_update_cols)
    ctx.qg_set_stream(bool(args.qg_stream))
    ctx.set_packet_streams(args.packet_streams)
    ctx.set_gather_mode(args.gather_mode)
    w = build_workload(ctx, args, lo, hi, n_total)
    ctx.packets_set(w["x"], w["k"])

    def barrier():
        if distributed:
            dist.barrier()

    progress("metric")
    elapsed, kms, launches, (clock_ghz, clock_spread) = timed(ctx, w, args, dev, args.steps, args.warmup, barrier)
    if distributed:
        elapsed = max_over_ranks(elapsed, backend=args.dist_backend)
    xg, kg = ctx.packets_get()
    finite = bool(np.isfinite(xg).all() and np.isfinite(kg).all())
    gathered = None
    if distributed and args.gather:
        # device-side gather of the trajectories (the frame writer's input): libswrt -> torch buffer -> all_gather
        full = gather_packets(ctx, n_total, world, rank)
        gathered = None if full is None else bool(np.isfinite(full[0]).all() and np.isfinite(full[1]).all()
                                                  and full[0].shape[0] == n_total)

    N = hi - lo
    ivs = w["intervals"]
    total_ps = n_total * args.substeps * ivs * args.steps
    value = total_ps / elapsed
    # sampled HIP-event time of the packet kernel; without samples fall back to wall time per step
    avg_launch_s = (kms / 1e3) / launches if launches > 0 else elapsed / args.steps
    spl = steps_per_launch_of(args, ivs)
    key = (f"{args.mode}_nx{args.nx}_N{N}_sub{args.substeps}" + (f"_iv{ivs}" if ivs > 1 else "")
           + ("_fma" if args.gather_mode == 1 else ""))
    pmc, pmc_note = (load_pmc(key) if args.kernel in (0, 2)
                     else (None, "PMC only for the default bit-exact tile kernel"))
    # Two packet streams: each launch is two half launches whose spans overlap
    # the neighbouring calls', so a launch's event span is not its share of
    # the GPU; the roofline then uses the wall time per launch of the timed
    # region (re-binning kernels and launch gaps included: a lower bound on
    # the kernel's own rate).  One stream: the HIP-event launch time.
    launches_per_step = max(1, -(-args.substeps * ivs // spl))
    two = args.packet_streams > 1 and args.kernel in (0, 2) and N >= 65536  # the library's kMultiStreamFrom
    basis_s = elapsed / (args.steps * launches_per_step) if two else avg_launch_s
    roof = roofline(pmc, N, args.nx, w["nslots"], spl, basis_s, launches, args.timing_every)
    roof["time_basis"] = (f"wall time per launch of the timed region ({args.packet_streams} overlapping part "
                          "launches per launch)"
                          if two else "HIP-event time of the packet-kernel launches")
    roof["launch_span_ms"] = avg_launch_s * 1e3
    roof["pmc_note"] = pmc_note
    add_observed_clock(roof, clock_ghz, clock_spread)
    workload = ("qg2layersw_raytrace packet loop (configs[3]): 2-layer QG, layer 1, "
                f"{'two-snapshot blend' if w['nslots'] == 2 else 'steady'}, {args.nx}^2x2 field, {n_total} packets "
                f"({args.scaling} scaling, {N} on rank 0's GPU), leapfrog dt {0.25 / args.substeps:g}*dx/U0 "
                f"({args.substeps} per PDE interval)" + (f", {ivs} PDE intervals per call" if ivs > 1 else ""))
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "packet-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,  # one step = `intervals` PDE intervals
        "higher_is_better": True,
        "scaling": args.scaling,
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": workload,
                   "nx": args.nx, "packets_total": n_total, "packets_per_gpu": N, "substeps_per_step": args.substeps,
                   "pde_dt": "0.25*dx/U0", "leapfrog_dt": f"{0.25 / args.substeps:g}*dx/U0",
                   "steps_per_launch": spl, "intervals_per_step": ivs,
                   "mode": args.mode, "rebin_every": args.rebin_every, "tile": args.tile, "kernel": args.kernel,
                   "sparse_tiles": args.sparse_tiles,
                   "packet_streams": args.packet_streams, "gather_mode": args.gather_mode,
                   "positions": args.positions, "field": args.field,
                   "parallelism": f"packets sharded x{world} ({args.scaling}), field replicated"},
        "roofline": roof,
        "finite": finite,
    }
    if gathered is not None:
        out["gathered_finite"] = gathered
    if not args.no_fma and args.kernel in (0, 2) and args.gather_mode == 0:
        # the opt-in FMA gather (tolerance parity, tests/test_gpu_parity.py::test_fma_gather_mode_tolerance):
        # the same workload and packets, timed the same way; the headline stays bit-exact
        progress("fma_gather")
        ctx.packets_set(w["x"], w["k"])
        ctx.set_gather_mode(1)
        el2, kms2, l2, (clk2, _) = timed(ctx, w, args, dev, args.steps, args.warmup, barrier)
        ctx.set_gather_mode(0)
        if distributed:
            el2 = max_over_ranks(el2, backend=args.dist_backend)
        ctx.packets_set(w["x"], w["k"])
        out["fma_gather"] = {"value": total_ps / el2, "ms_per_step": el2 / args.steps * 1e3,
                             "avg_launch_ms": (kms2 / l2) if l2 else None, "vs_exact": elapsed / el2,
                             "clock_ghz_observed": clk2,
                             "parity": "tolerance: stencil sums and blend by fused multiply-add, "
                                       "<= 1e-13 relative per step vs the bit-exact path"}
    if world == 1 and not args.no_forecast and args.scaling == "strong":
        progress("strong_scaling_forecast")
        out["strong_scaling_forecast"] = strong_scaling_forecast(ctx, w, args, dev, n_total, value)
        if args.forecast_intervals > 1 and w["nslots"] == 2 and args.kernel in (0, 2):
            out["strong_scaling_forecast_intervals"] = intervals_forecast(ctx, w, args, dev, n_total, value,
                                                                          args.forecast_intervals)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the GPU box's CPU share for one GPU is 16 threads (OMP_NUM_THREADS there)
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
        progress("cpu_baseline")
        out["cpu_baseline"] = cpu_baseline(ctx, w, args.cpu_seconds, threads)
        # all host cores (every CPU this process may run on) and 1 core
        try:
            allc = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            allc = os.cpu_count() or 1
        if allc != threads:
            out["cpu_baseline_all_cores"] = cpu_baseline(ctx, w, args.cpu_seconds * 2 / 3, allc)
            out["cpu_baseline_all_cores"]["note"] = (
                f"{allc} OpenMP threads = every CPU this process may run on; the job's cgroup CPU quota "
                f"({host_cpu()['cgroup_cpu_quota']} cores) caps them, so cpu_baseline's {threads} threads is the "
                f"faster figure on this box")
        out["cpu_baseline_1core"] = cpu_baseline(ctx, w, args.cpu_seconds / 3, 1)
    elif rank == 0:
        out["cpu_baseline"] = None
    if args.driver_steps > 0 and args.mode == "blend":
        progress("driver_step")
        out["driver_step"] = driver_step(ctx, w, args, dev, distributed, n_total)
        if world == 1 and not args.no_forecast and args.scaling == "strong":
            progress("driver_step_forecast")
            fc = driver_forecast(ctx, w, args, dev, n_total, out["driver_step"])
            pk = out.get("strong_scaling_forecast", {})
            for G in ("2", "4", "8"):
                if G in pk:  # packets alone at this shard (the metric's form) vs the PDE alone
                    fc[G]["packets_alone_ms"] = pk[G]["ms_per_step"]
                    fc[G]["bound"] = "pde" if fc["pde_alone_ms"] > pk[G]["ms_per_step"] else "packets"
            progress("driver_step_forecast owner")
            fc["owner"] = owner_forecast(ctx, w, args, dev, n_total, out["driver_step"]["ms_per_pde_step"])
            out["driver_step_forecast"] = fc
    if args.ode23_steps > 0 and args.mode == "blend" and world == 1:
        # (single rank: a sharded ode23 needs the error norm's allreduce, PacketEnsemble(shard=...))
        progress("driver_step_ode23")
        out["driver_step_ode23"] = driver_step(ctx, w, args, dev, distributed, n_total, integrator="ode23",
                                               nsteps=args.ode23_steps)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if distributed:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
