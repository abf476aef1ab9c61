"""Tracing packets through a stored PV series (BASELINE configs[2],
"Time-evolving QG snapshots (read_field)").

The reference's stored-field consumer reads PV frames written by the
drivers (``symplectic_full_fourier.m:18-20``: ``read_field("analysis/pv",
nx, nx, 1, [2000])`` then ``k2g(-g2k(q)./(K_d2+K2))``).  Here every frame of
a ``pv.bin`` series (``read_field.m:37-98``: headerless fp64 frames of
nx x nx [x nlayers]) goes to the GPU once, ``g2k`` and ``grid_U``
(``g2k.m:8-9``, ``grid_U.m:1-18``) run there into a packet slot
(``swrt_set_field_q``), and the packets advance through consecutive frame
pairs [t_i, t_{i+1}] with interpolate_U's linear blend
(``interpolate_U.m:19-23``) by ``nsub`` fused leapfrog substeps per
interval, up to four intervals per call (``swrt_advance_intervals``: the
same bits as one call per interval).
"""
from __future__ import annotations

import math
import os

import numpy as np

from ._lib import Context
from .integrate import PacketEnsemble
from .io import read_field
from .scheme import BUMP_QG

SLOT_INTERVALS = 4  # SWRT_MAX_SLOTS - 1 intervals per swrt_advance_intervals call


def frame_count(pv_path, nx, nlayers=1):
    """Frames in ``pv_path``.bin (read_field.m:60-66: file size / frame size)."""
    return os.path.getsize(str(pv_path) + ".bin") // (8 * nx * nx * nlayers)


def read_frame(pv_path, nx, frame, nlayers=1):
    """read_field(pv, nx, nx, nlayers, frame) for one frame (1-based), read
    by offset so a long series is never loaded whole: (nx, nx[, nlayers])."""
    per = nx * nx * nlayers
    a = np.fromfile(str(pv_path) + ".bin", dtype=np.float64, count=per, offset=8 * per * (int(frame) - 1))
    if a.size != per:
        raise ValueError(f"{pv_path}.bin has no frame {frame}")
    a = a.reshape((nx, nx, nlayers), order="F")
    return a[:, :, 0] if nlayers == 1 else a


def trace_stored(pv_path, nx, x, k, f, Cg, *, frames=None, times=None, nlayers=1, L=2 * math.pi, K_d2=None,
                 shear=0.0, k_scale=1.0, nsub=5, bump=BUMP_QG, out_dir=None, intervals_per_call=SLOT_INTERVALS,
                 ctx: Context | None = None, shard=None):
    """Advance packets (x, k: N x 2) through the stored frames of a PV series.

    ``frames``: 1-based frame numbers in time order (default: every frame in
    the file).  ``times``: the frames' times (default: ``pv_time.bin`` next to
    ``pv_path``, as written by write_field beside pv.bin,
    qgsw_raytrace.m:108-109,170-171).  ``nlayers`` = 2 reads 2-layer frames
    and traces through layer 1 with interpolate's 2*nx y-period (the 2-layer
    driver's semantics, qg2layersw_raytrace.m:186-188); ``L``, ``K_d2``
    (default f/Cg), ``shear``, ``k_scale`` are grid_U's.  ``out_dir``: write
    packet_x/k/time.bin frames (write_field layout) at the first frame and
    after every call.  Returns (x, k, t_end)."""
    ctx = ctx if ctx is not None else Context(0)
    nx = int(nx)
    if frames is None:
        frames = list(range(1, frame_count(pv_path, nx, nlayers) + 1))
    frames = [int(fr) for fr in frames]
    if len(frames) < 2:
        raise ValueError("need at least two frames")
    if times is None:
        tp = os.path.join(os.path.dirname(str(pv_path)) or ".", "pv_time")
        tall = read_field(tp)[0]
        times = [float(tall[fr - 1]) for fr in frames]
    times = [float(t) for t in times]
    if len(times) != len(frames) or any(b <= a for a, b in zip(times, times[1:])):
        raise ValueError("times must match frames and increase")
    K_d2 = f / Cg if K_d2 is None else K_d2
    ny_period = nx * nlayers
    intervals_per_call = max(1, min(int(intervals_per_call), SLOT_INTERVALS))

    def load(slot, fr):
        q = read_frame(pv_path, nx, fr, nlayers)
        ctx.set_field_q(slot, q if nlayers == 1 else q[:, :, 0], L, K_d2, shear, k_scale, ny_period)

    ens = PacketEnsemble(x, k, L, f, Cg, nx, K_d2, shear=shear, k_scale=k_scale, nlayers=nlayers, bump=bump,
                         ctx=ctx, shard=shard)
    if out_dir is not None:
        os.makedirs(out_dir, exist_ok=True)
        ens.write_frame(times[0], out_dir)
    load(0, frames[0])
    i = 1
    while i < len(frames):
        g = min(intervals_per_call, len(frames) - i)
        for j in range(g):
            load(1 + j, frames[i + j])
        ens.advance_intervals([times[i + j] - times[i + j - 1] for j in range(g)], nsub)
        ctx.swap_slots(0, g)  # the last frame starts the next call
        i += g
        if out_dir is not None:
            ens.write_frame(times[i - 1], out_dir)
    xs, ks = ens.state()
    return xs, ks, times[-1]
