"""run.log in the layout the reference's consumers parse.

The reference drivers print their parameter block with ``fprintf``
(``qgsw_raytrace.m:76-88``, ``qg2layersw_raytrace.m:85-97``) into the SLURM
job log of ``matlab -nodisplay -r ...`` (``runqgsw_raytrace.sbatch:31``), so
every run.log starts with the 10 lines MATLAB's banner occupies
(``analysis/job-37011720/run-16/run.log:1-10``) and the block starts on
line 11.  Both consumers rely on that offset: ``analysis/load_data.m:18-22``
and ``symplectic_full_fourier.m:72-76`` call
``textscan(fid, 'Resolution: %dx%d', 1, ..., 'headerlines', 10)`` and then
``headerlines 7`` to reach ``Coriolis parameter``.  :class:`RunLog` writes
the same 10-line preamble (this library's banner in the banner's place), the
block, the ``Simulation progress`` lines every 51 steps
(``qgsw_raytrace.m:119,173-175``) and ``Real time elapsed``
(``qgsw_raytrace.m:177-179``, ``qg2layersw_raytrace.m:244-246``).
"""
from __future__ import annotations

import datetime
import time

PREAMBLE_LINES = 10   # analysis/load_data.m:18 'headerlines', 10


def preamble():
    """Ten lines standing where ``matlab -nodisplay`` prints its banner."""
    when = datetime.datetime.now().strftime("%B %d, %Y")
    lines = [
        "",
        " " * 26 + "< s w r t : wave-packet ray tracing on MI355X >",
        " " * 26 + "swraytracing_amd (libswrt, gfx950 HIP, fp64)",
        " " * 26 + when,
        "",
        " ",
        "The parameter block starts on line 11, as in a `matlab -nodisplay` job log:",
        "analysis/load_data.m:18 and symplectic_full_fourier.m:72 skip 10 header lines.",
        " ",
        " ",
    ]
    assert len(lines) == PREAMBLE_LINES
    return "\n".join(lines) + "\n"


def parameter_block(nx, Npackets, wavenumber_radius, dt, T, spin_up, steps_per_save, packet_steps_per_save,
                    f, Cg, U_g, U0, Fr, K_d2, two_layer=False):
    """qgsw_raytrace.m:76-88 / qg2layersw_raytrace.m:85-97, MATLAB's %d / %f."""
    return "".join([
        f"Resolution: {nx}x{nx}\n",
        f"Number of packets: {Npackets}\n",
        f"Initial wavenumber radius: {wavenumber_radius:f}\n",
        (f"Initial time step: {dt:f}\n" if two_layer else f"Time step: {dt:f}\n"),
        f"Simulation time: {T:f}\n",
        f"Spin-up time: {spin_up:f}\n",
        f"Steps per save: {steps_per_save}\n",
        f"Steps per packet save: {packet_steps_per_save}\n",
        f"Coriolis parameter: {f:f}\n",
        f"Group velocity: {Cg:f}\n",
        f"Background velocity (parameter,computed): ({U_g:f},{U0:f})\n",
        f"Froude Number: {Fr:f}\n",
        f"Deformation wavenumber: {K_d2:f}\n",
    ])


class RunLog:
    """The driver's log (``create_logger``, qgsw_raytrace.m:182-189, qg2layersw_raytrace.m:249-256): every
    message goes to ``path`` (rank 0 of a sharded run; None: no file) and,
    when ``verbose``, to stdout.  The file starts with :func:`preamble`."""

    def __init__(self, path, verbose=False):
        self.f = open(path, "w") if path else None
        self.verbose = verbose
        self.t0 = None
        if self.f:
            self.f.write(preamble())
            self.f.flush()

    def __call__(self, msg):
        if self.verbose:
            print(msg, end="")
        if self.f:
            self.f.write(msg)
            self.f.flush()

    def start(self):
        """tic + 'Simulation progress:  0.00%' (qgsw_raytrace.m:114,119)."""
        self.t0 = time.perf_counter()
        self("Simulation progress:  0.00%")

    def progress(self, step, Nsteps):
        """qgsw_raytrace.m:173-175: every 51 steps, '% 6.2f%%\\n'."""
        if step % 51 == 0:
            self(f"{step / Nsteps * 100: 6.2f}%\n")

    def finish(self):
        """qgsw_raytrace.m:177-179: '100.00%' and the toc line."""
        self("100.00%\n")
        el = time.perf_counter() - self.t0 if self.t0 is not None else 0.0
        self(f"Real time elapsed: {el:.3f} seconds\n")

    def close(self):
        if self.f:
            self.f.close()
            self.f = None
