"""Config 5 (BASELINE.json configs[4]) fp32 tolerance study: the exact
spectral evaluator on a 1024^2 field (symplectic_full_fourier.m: scheme from
the streamfunction, ode_symplectic with dt = 0.1*dx/max(Cg, U0), f = 3,
gH = 1), a strided subset of the 1e7-packet ensemble, fp32 and fp64 leapfrog
side by side.  Per checkpoint: max |x32 - x64|, max |k32 - k64| / max|k|, and
the absolute-frequency drift |Omega_abs - Omega_0| / Omega_0 of both runs
(symplectic_full_fourier.m:41,54-57; Omega_abs evaluated in fp64).  Prints one
JSON object (the table committed under profiles/).  tests/test_gpu_spectral.py
asserts the envelope on a smaller subset."""
import argparse
import json
import os
import sys

import numpy as np
import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import swraytracing_amd as sw  # noqa: E402


def spectrum(nx, seed=146, amp=0.05):
    """|psi_k| ~ |k|^-3 random phases, 1 <= |k| <= 0.75 kmax."""
    kmax = nx // 2 - 1
    rng = np.random.default_rng(seed)
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(kmax + 1)[None, :]
    kk = np.sqrt(kx * kx + ky * ky)
    mask = (kk >= 1) & (kk <= 0.75 * kmax)
    psik = np.zeros((2 * kmax + 1, kmax + 1), complex)
    psik[mask] = kk[mask] ** -3.0 * np.exp(2j * np.pi * rng.random(mask.sum()))
    return psik * amp


def ensemble_subset(ntot, stride, L, seed=123):
    """Every `stride`-th packet of the ntot ensemble of symplectic_full_fourier.m:24-28
    (k = 3 [cos, sin](2 pi i / N), x uniform in [-L/2, L/2))."""
    i = np.arange(1, ntot + 1, stride, dtype=np.float64)
    k = 3.0 * np.stack([np.cos(2 * np.pi * i / ntot), np.sin(2 * np.pi * i / ntot)], axis=1)
    x = L * np.random.default_rng(seed).random((i.size, 2)) - L / 2
    return x, k


def omega_abs(sch, x, k, f, gH):
    sch.precision = 64
    _, I = sch._eval(x)
    return np.sqrt(f * f + gH * (k * k).sum(1)) + I[0] * k[:, 0] + I[1] * k[:, 1]


def study(ctx, nx=1024, ntot=10_000_000, stride=153, chunks=8, per_chunk=8, f=3.0, Cg=1.0):
    L = 2 * np.pi
    dx = L / nx
    sch = sw.FourierScheme.from_halfplane(spectrum(nx), ctx=ctx)
    g = np.linspace(0, L, 256, endpoint=False)
    XX, YY = np.meshgrid(g, g)
    sch.precision = 64
    _, Ig = sch._eval(np.stack([XX.ravel(), YY.ravel()], axis=1))
    U0 = float(np.sqrt(Ig[0] ** 2 + Ig[1] ** 2).max())
    dt = 0.1 * dx / max(Cg, U0)  # symplectic_full_fourier.m:37
    gH = Cg ** 2
    x0, k0 = ensemble_subset(ntot, stride, L)
    # fp32 evaluation error of U and grad U at the start points
    _, I64 = sch._eval(x0)
    sch.precision = 32
    _, I32 = sch._eval(x0)
    eU = float(np.abs(I32[0:2] - I64[0:2]).max())
    eG = float(np.abs(I32[2:6] - I64[2:6]).max())
    Om0 = omega_abs(sch, x0, k0, f, gH)
    st = {64: (x0.copy(), k0.copy()), 32: (x0.copy(), k0.copy())}
    rows = []
    for c in range(chunks):
        for prec in (64, 32):
            sch.precision = prec
            st[prec] = sch.leapfrog(st[prec][0], st[prec][1], dt, per_chunk, f, gH)
        (x6, k6), (x3, k3) = st[64], st[32]
        rows.append({"steps": (c + 1) * per_chunk,
                     "max_abs_x_err": float(np.abs(x3 - x6).max()),
                     "max_rel_k_err": float(np.abs(k3 - k6).max() / np.abs(k6).max()),
                     "omega_abs_drift_fp64": float((np.abs(omega_abs(sch, x6, k6, f, gH) - Om0) / Om0).max()),
                     "omega_abs_drift_fp32": float((np.abs(omega_abs(sch, x3, k3, f, gH) - Om0) / Om0).max())})
    return {"nx": nx, "packets": int(x0.shape[0]), "subset_of": ntot, "stride": stride, "dt": dt, "dx": dx,
            "U0": U0, "f": f, "gH": gH, "fp32_eval_err_U": eU, "fp32_eval_err_gradU": eG, "table": rows}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--stride", type=int, default=39)  # 256,411 of the 1e7 packets
    ap.add_argument("--chunks", type=int, default=16)
    ap.add_argument("--per-chunk", type=int, default=16)
    a = ap.parse_args()
    ctx = sw.Context(0)
    out = study(ctx, a.nx, stride=a.stride, chunks=a.chunks, per_chunk=a.per_chunk)
    out["what"] = "config 5 fp32 tolerance study (tools/fp32_study.py)"
    print(json.dumps(out))
    ctx.close()


if __name__ == "__main__":
    main()
