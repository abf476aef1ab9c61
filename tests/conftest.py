import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import cbind
    cbind.build()
    return cbind


@pytest.fixture(scope="session")
def ctx():
    """One device context for the whole GPU session (one process on the GPU)."""
    import swraytracing_amd as sw
    c = sw.Context(0)
    yield c
    c.close()


@pytest.fixture()
def fresh_ctx():
    """A device context of its own for one test.  The session context may
    carry a QG stream from an earlier driver test; while one is initialised
    every advance call joins the extra packet streams at its end
    (slot_events), so split launches never overlap across calls there — the
    packet-stream tests and the bench-configuration tests need the bench's own
    state (no QG stream)."""
    import swraytracing_amd as sw
    c = sw.Context(0)
    yield c
    c.close()


def periodic_grid(nx, L=2 * np.pi):
    xs = np.arange(nx) * (L / nx)
    return np.meshgrid(xs, xs, indexing="ij")


@pytest.fixture(scope="session")
def qg_case():
    """Small single-layer QG background (qgsw_raytrace.m setup) + packets."""
    from oracle import swrt_oracle as orc
    nx, L, f, Cg, Ug, w0 = 64, 2 * np.pi, 3.0, 1.0, 0.2, 4.0
    rng = np.random.default_rng(146)
    K_d2 = f / Cg
    q = orc.initial_q(nx, L, Ug, K_d2, 5, 8, rng)
    kx_, ky_, K2 = orc.wavenumber_grids(nx)
    qk = orc.g2k(q)
    flow = orc.grid_U(qk, K_d2, K2, kx_, ky_)
    x, k = orc.initial_packets(256, L, w0, f, Cg, rng)
    speed = np.sqrt(flow["u"] ** 2 + flow["v"] ** 2).max()
    dt = 0.05 * (L / nx) / speed
    return dict(nx=nx, L=L, f=f, Cg=Cg, K_d2=K_d2, q=q, qk=qk, flow=flow, x=x, k=k, dt=dt,
                kx_=kx_, ky_=ky_, K2=K2)
