"""ctypes binding of the C oracle (oracle/build/libswrt_oracle.so).

TEST INFRASTRUCTURE ONLY — used by tests/ and bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libswrt_oracle.so")
_lib = None

_D = ctypes.c_double
_I = ctypes.c_int64
_P = ctypes.POINTER(ctypes.c_double)


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_eval.argtypes = [_P, _P, _D, _I, _D, _D, _D, _P, _P, _I, _P]
        L.oracle_eval.restype = None
        L.oracle_leapfrog.argtypes = [_P, _P, _D, _D, _I, _D, _D, _D, _P, _P, _I, _D, _I, _D, _D,
                                      _I, _P, _P]
        L.oracle_leapfrog.restype = None
        _bind_fast(L)
        L.oracle_num_threads.restype = ctypes.c_int
        L.oracle_set_threads.argtypes = [ctypes.c_int]
        L.oracle_set_threads.restype = None
        _lib = L
    return _lib


_CPU_FLAGS = ["-O3", "-march=native", "-fopenmp", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-std=c11"]


def cpu_lib(out_dir):
    """The oracle compiled for THIS host's CPU (-O3 -march=native, no FMA
    contraction: the same bits) into out_dir — bench.py's cpu_baseline build,
    compiled where it runs so -march=native means that machine.  Returns
    (ctypes lib, flags string)."""
    os.makedirs(out_dir, exist_ok=True)
    path = os.path.join(out_dir, "libswrt_oracle_cpu.so")
    subprocess.run(["gcc"] + _CPU_FLAGS + ["-shared", "-o", path, os.path.join(_HERE, "swrt_oracle.c"), "-lm"],
                   check=True)
    L = ctypes.CDLL(path)
    _bind_fast(L)
    L.oracle_num_threads.restype = ctypes.c_int
    L.oracle_set_threads.argtypes = [ctypes.c_int]
    L.oracle_set_threads.restype = None
    return L, "gcc " + " ".join(_CPU_FLAGS)


def _bind_fast(L):
    L.oracle_leapfrog_fast.argtypes = [_P, _P, _D, _D, _I, _D, _D, _D, _P, _P, _I, _D, _I, _D, _D]
    L.oracle_leapfrog_fast.restype = None


def leapfrog_fast(planes0, planes1, alpha0, dalpha, nx, nyF, dx, bump, x, k, dt, nsteps, f, gH, L=None):
    """oracle_leapfrog_fast (CPU-arranged, same bits as leapfrog): -> (x, k)."""
    L = L or lib()
    x = np.asfortranarray(x, dtype=np.float64).copy(order="F")
    k = np.asfortranarray(k, dtype=np.float64).copy(order="F")
    L.oracle_leapfrog_fast(_ptr(planes0), _ptr(planes1), alpha0, dalpha, nx, float(nyF), dx, bump,
                           x.ctypes.data_as(_P), k.ctypes.data_as(_P), x.shape[0], dt, nsteps, f, gH)
    return x, k


def _ptr(a):
    return a.ctypes.data_as(_P) if a is not None else None


def planes_of(fields):
    """dict of 6 grids (u,v,ux,uy,vx,vy) -> contiguous 6 x nx*nx column-major planes."""
    from .swrt_oracle import FIELD_ORDER  # noqa: E402  (package-relative when imported as oracle.cbind)
    return np.ascontiguousarray(np.stack([np.asarray(fields[n], dtype=np.float64).ravel(order="F")
                                          for n in FIELD_ORDER]))


def eval6(planes0, planes1, alpha, nx, nyF, dx, bump, x, y):
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    out = np.empty((6, x.size))
    lib().oracle_eval(_ptr(planes0), _ptr(planes1), alpha, nx, float(nyF), dx, bump, _ptr(x), _ptr(y),
                      x.size, _ptr(out))
    return out


def leapfrog(planes0, planes1, alpha0, dalpha, nx, nyF, dx, bump, x, k, dt, nsteps, f, gH,
             save_every=0):
    """State x, k: N x 2 (any order) -> returns new (x, k) N x 2 and history frames."""
    x = np.asfortranarray(x, dtype=np.float64).copy(order="F")
    k = np.asfortranarray(k, dtype=np.float64).copy(order="F")
    n = x.shape[0]
    nfr = nsteps // save_every if save_every else 0
    hx = np.empty((nfr, 2, n)) if nfr else None
    hk = np.empty((nfr, 2, n)) if nfr else None
    lib().oracle_leapfrog(_ptr(planes0), _ptr(planes1), alpha0, dalpha, nx, float(nyF), dx, bump,
                          x.ctypes.data_as(_P), k.ctypes.data_as(_P), n, dt, nsteps, f, gH,
                          save_every if nfr else 0, _ptr(hx), _ptr(hk))
    return x, k, hx, hk


def raytracing_rhs(planes0, planes1, f, Cg, tmax, nx, nyF, dx, bump):
    """odefun of qgsw_raytrace.m:258-268 (the restatement swrt_oracle.
    raytracing_rhs) with interpolate_U by oracle_eval (OpenMP): the same
    operations in the same order, so the same bits — tests check that on a
    subset before relying on it for large ensembles."""
    def odefun(t, y):
        n = y.size // 4
        e = eval6(planes0, planes1, t / tmax, nx, nyF, dx, bump, y[0:n], y[n:2 * n])
        k1, k2 = y[2 * n:3 * n], y[3 * n:4 * n]
        s = np.sqrt(f**2 + Cg**2 * (k1 * k1 + k2 * k2))
        dx1 = e[0] + (Cg * k1) / s
        dx2 = e[1] + (Cg * k2) / s
        dk1 = -(e[2] * k1 + e[4] * k2)
        dk2 = -(e[3] * k1 + e[5] * k2)
        return np.concatenate([dx1, dx2, dk1, dk2])
    return odefun
