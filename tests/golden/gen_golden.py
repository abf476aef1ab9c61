"""Generate the committed golden fixtures from the numpy oracle.

The MATLAB reference cannot run here and ships no numeric vectors, so these
fixtures are produced by the CPU restatement (oracle/swrt_oracle.py), which
tests/test_oracle_kats.py pins against analytic known answers.  Re-run with
`python tests/golden/gen_golden.py` (deterministic: numpy PCG64 seeds).
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import swrt_oracle as orc  # noqa: E402


def planes(flow):
    return np.stack([np.asarray(flow[n]).ravel(order="F") for n in orc.FIELD_ORDER])


def qg_fixture():
    nx = 32
    rng = np.random.default_rng(2718)
    q = orc.initial_q(nx, 2 * np.pi, 0.2, 3.0, 5, 8, rng)
    qk1 = orc.g2k(q)
    m1 = orc.QG1Oracle(qk1, nx, 3.0, r_drag=0.0, force_strength=0.1, f=3.0, Cg=1.0, use_filter=True)
    dt1 = 0.05 * (2 * np.pi / nx) / 0.2
    for _ in range(8):
        m1.step(dt1)
    q2 = orc.initial_q(nx, 20.0, 0.2, 3.0, 1, 3, rng)
    qk2 = np.stack([orc.g2k(q2), orc.g2k(-q2)], axis=2)
    m2 = orc.QG2Oracle(qk2, nx, 20.0, 3.0, shear_strength=0.5)
    dts = []
    for _ in range(8):
        m2.step()
        dts.append(m2.dt)
    return dict(nx=nx, qk1_0=qk1, qk1_8=m1.qk, dt1=dt1, qk2_0=qk2, qk2_8=m2.qk, dts2=np.array(dts),
                L2=20.0, K_d2=3.0, f=3.0, Cg=1.0)


def main():
    nx, L, f, Cg = 32, 2 * np.pi, 3.0, 1.0
    rng = np.random.default_rng(146)
    K_d2 = f / Cg
    q = orc.initial_q(nx, L, 0.2, K_d2, 5, 8, rng)
    kx_, ky_, K2 = orc.wavenumber_grids(nx)
    qk = orc.g2k(q)
    flow = orc.grid_U(qk, K_d2, K2, kx_, ky_)
    x, k = orc.initial_packets(64, L, 4.0, f, Cg, rng)
    # include cell-edge / wrap edge cases
    dx = L / nx
    x[0] = [0.0, 0.0]
    x[1] = [-1e-17, L]
    x[2] = [5 * dx, -7 * dx]
    x[3] = [-L / 2, L / 2]
    speed = np.sqrt(flow["u"] ** 2 + flow["v"] ** 2).max()
    dt = 0.05 * dx / speed
    # steady (SpectralScheme path, bump 1e-13)
    snap = orc.GridField(flow, dx)
    xs, ks, hx, hk = orc.leapfrog(x, k, dt, 40, f, Cg**2, snap, bump=orc.BUMP_SW, save_every=10)
    np.savez_compressed(os.path.join(HERE, "golden_steady.npz"), planes=planes(flow), nx=nx, L=L, f=f, gH=Cg**2,
                        dt=dt, nsteps=40, save_every=10, bump=orc.BUMP_SW, x0=x, k0=k, x=xs, k=ks,
                        hist_x=np.stack(hx), hist_k=np.stack(hk))
    # two snapshots, 2-layer y-period, bump 1e-10
    q2 = orc.initial_q(nx, L, 0.2, K_d2, 5, 8, rng)
    flow2 = orc.grid_U(orc.g2k(0.8 * q + 0.2 * q2), K_d2, K2, kx_, ky_, 0.5)
    flow1 = orc.grid_U(qk, K_d2, K2, kx_, ky_, 0.5)
    s1 = orc.GridField(flow1, dx, 2 * nx)
    s2 = orc.GridField(flow2, dx, 2 * nx)
    xb, kb, _, _ = orc.leapfrog(x, k, dt, 16, f, Cg**2, s1, s2, alpha0=1 / 32, dalpha=1 / 16, bump=orc.BUMP_QG)
    np.savez_compressed(os.path.join(HERE, "golden_blend.npz"), planes0=planes(flow1), planes1=planes(flow2),
                        nx=nx, ny_period=2 * nx, L=L, f=f, gH=Cg**2, dt=dt, nsteps=16, alpha0=1 / 32,
                        dalpha=1 / 16, bump=orc.BUMP_QG, x0=x, k0=k, x=xb, k=kb)
    # field preparation (SpectralScheme ctor, grid_U) — FFT round-off tolerance
    psi = orc.k2g(-qk / (K_d2 + K2))
    sf = orc.spectral_scheme_fields(L, nx, psi)
    np.savez_compressed(os.path.join(HERE, "golden_fields.npz"), psi_in=psi, psi=sf["psi"],
                        planes_psi=planes(sf), qk=qk, K_d2=K_d2, planes_qk=planes(flow),
                        planes_qk_shear=planes(flow1))
    # QG PDE steppers (qgsw_raytrace.m:111-137 / qg2layersw_raytrace.m:129-181)
    qg = qg_fixture()
    np.savez_compressed(os.path.join(HERE, "golden_qg.npz"), **qg)
    # ode23 over the blend fixture's snapshots (qgsw_raytrace.m:143-150)
    T = 12 * dt
    rhs = orc.raytracing_rhs({n: flow1[n] for n in orc.FIELD_ORDER}, {n: flow2[n] for n in orc.FIELD_ORDER},
                             f, Cg, T, dx, nyF=2 * nx)
    y0 = np.concatenate([x[:, 0], x[:, 1], k[:, 0], k[:, 1]])
    st = {}
    ts, yT = orc.ode23(rhs, [0.0, T], y0, stats=st)
    np.savez_compressed(os.path.join(HERE, "golden_ode23.npz"), planes0=planes(flow1), planes1=planes(flow2),
                        nx=nx, ny_period=2 * nx, L=L, f=f, Cg=Cg, tmax=T, x0=x, k0=k, ts=ts, y=yT,
                        failed=st["failed"])
    for fn in ("golden_steady.npz", "golden_blend.npz", "golden_fields.npz", "golden_qg.npz",
               "golden_ode23.npz"):
        print(fn, os.path.getsize(os.path.join(HERE, fn)))


if __name__ == "__main__":
    main()
