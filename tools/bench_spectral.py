"""Config 5 study (BASELINE.json configs[4]): exact spectral evaluator on a
1024^2 spectral field, fp64 vs fp32 — throughput, FP roofline and the fp32
error growth.  Prints one JSON line.  Not the driver's bench (bench.py is).

Accounting: F = 22 flop x M modes per packet-step (M = the modes inside the
rows' nonzero spans, which the kernel sums): per mode and lane 5 mul + 7 FMA
+ 3 add (z = C*e, the five row sums, the phase recurrence, kx += ds) — the
instructions of swrt_spectral.hpp's inner loop (SURVEY §8d E2 counted 16).
Peaks: FP64 vector 78.6 TFLOP/s, FP32 vector 157.3 TFLOP/s (packed; MI355X
spec, MI355X_MICROARCH.md chip table).  The rate includes the host copies of
the call; the kernels' VALU-issue fractions from PMC are tools/pmc_rows.sh's."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import swraytracing_amd as sw  # noqa: E402

PEAK = {64: 78.6, 32: 157.3}
FLOP_PER_MODE = 22


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nx", type=int, default=1024)
    ap.add_argument("--packets", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=2)
    args = ap.parse_args()
    nx = args.nx
    kmax = nx // 2 - 1
    rng = np.random.default_rng(146)
    # broadband random-phase spectrum |psi_k| ~ |k|^-3 for 1 <= |k| <= 0.75 kmax
    kx = np.arange(-kmax, kmax + 1)[:, None]
    ky = np.arange(kmax + 1)[None, :]
    kk = np.sqrt(kx * kx + ky * ky)
    mask = (kk >= 1) & (kk <= 0.75 * kmax)
    psik = np.zeros((2 * kmax + 1, kmax + 1), complex)
    psik[mask] = kk[mask] ** -3.0 * np.exp(2j * np.pi * rng.random(mask.sum()))
    sch = sw.FourierScheme.from_halfplane(psik * 0.05)
    M = (2 * kmax + 1) * (kmax + 1)
    # coefficients the kernel actually sums (nonzero span of every row)
    C = 2 * psik * 0.05
    nz = np.abs(C) > 0
    spans = [(np.flatnonzero(nz[:, j]).max() - np.flatnonzero(nz[:, j]).min() + 1) if nz[:, j].any() else 0
             for j in range(C.shape[1])]
    M_active = int(sum(spans))
    N = args.packets
    L = 2 * np.pi
    x = L * rng.random((N, 2)) - L / 2
    th = 2 * np.pi * np.arange(1, N + 1) / N
    k = np.sqrt(15.0) * 3.0 * np.stack([np.cos(th), np.sin(th)], axis=1)
    dt = 0.1 * (L / nx)
    res = {}
    for prec in (64, 32):
        sch.precision = prec
        sch.leapfrog(x[:256], k[:256], dt, 1, 3.0, 1.0)  # warm-up
        t0 = time.perf_counter()
        xs, ks = sch.leapfrog(x, k, dt, args.steps, 3.0, 1.0)
        t = time.perf_counter() - t0
        rate = N * args.steps / t
        tf = rate * FLOP_PER_MODE * M_active / 1e12
        res[prec] = dict(x=xs, k=ks, rate=rate, tflops=tf, seconds=t)
    err = float(np.abs(res[32]["x"] - res[64]["x"]).max())
    errk = float(np.abs(res[32]["k"] - res[64]["k"]).max() / np.abs(res[64]["k"]).max())
    out = {
        "metric": "packet-steps/sec, exact spectral evaluator (config 5 study)",
        "config": {"workload": "symplectic_full_fourier path, exact Fourier-mode kick", "nx": nx,
                   "modes_dense": M, "modes_summed": M_active, "packets": N, "steps": args.steps},
        "fp64": {"value": res[64]["rate"], "unit": "packet-steps/s",
                 "roofline": {"bound": "valu-fp64", "achieved": res[64]["tflops"], "peak": PEAK[64],
                              "unit": "TFLOP/s", "frac": res[64]["tflops"] / PEAK[64]}},
        "fp32": {"value": res[32]["rate"], "unit": "packet-steps/s",
                 "roofline": {"bound": "valu-fp32", "achieved": res[32]["tflops"], "peak": PEAK[32],
                              "unit": "TFLOP/s", "frac": res[32]["tflops"] / PEAK[32]},
                 "max_abs_x_err_vs_fp64": err, "max_rel_k_err_vs_fp64": errk},
        "note": "host-buffer call incl. upload/download; 22 flop per summed mode (zero row ends skipped)",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
