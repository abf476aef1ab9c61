"""ctypes binding of libswrt.so (the C ABI in include/swrt.h).

There is no CPU fallback: if the HIP library is missing or the device call
fails, the error propagates.  Build it with
``python -c "import __graft_entry__ as g; g.build()"`` (hipcc, gfx950).
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

# One HIP runtime per process: torch wheels ship their own libamdhip64.so.7.
# Import torch (if present) before dlopen-ing libswrt so that our NEEDED
# libamdhip64.so.7 resolves to the runtime torch already loaded, instead of a
# second copy from /opt/rocm.
try:  # pragma: no cover - import side effect only
    import torch  # noqa: F401
except Exception:  # torch absent: the system HIP runtime is used
    pass

_HERE = os.path.dirname(os.path.abspath(__file__))
# SWRT_LIB_PATH: alternative build of the same ABI (tuning experiments only)
LIB_PATH = os.environ.get("SWRT_LIB_PATH") or os.path.join(_HERE, "libswrt.so")

SWRT_OK = 0
ERRORS = {1: "SWRT_ERR_ARG", 2: "SWRT_ERR_HIP", 3: "SWRT_ERR_STATE", 4: "SWRT_ERR_ALLOC"}

_D = ctypes.c_double
_I = ctypes.c_int64
_INT = ctypes.c_int
_P = ctypes.POINTER(ctypes.c_double)
_VP = ctypes.c_void_p
_HOOK = ctypes.CFUNCTYPE(None, ctypes.c_void_p)  # void (*)(void*)
_REDUCE = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.POINTER(ctypes.c_double), ctypes.c_void_p)  # int (*)(double*, void*)

class QGParams(ctypes.Structure):
    """swrt_qg_params (include/swrt.h)."""
    _fields_ = [("nlayers", ctypes.c_int), ("filter", ctypes.c_int), ("L", _D), ("K_d2", _D), ("beta", _D),
                ("r_drag", _D), ("force_strength", _D), ("f", _D), ("Cg", _D), ("shear", _D), ("nu", _D),
                ("hyper_order", _D), ("r", _D)]


# name -> (restype, argtypes).  Kept in the order of include/swrt.h.
SIGNATURES = {
    "swrt_version": (_INT, []),
    "swrt_create": (_INT, [_INT, ctypes.POINTER(_VP)]),
    "swrt_destroy": (None, [_VP]),
    "swrt_last_error": (ctypes.c_char_p, [_VP]),
    "swrt_set_field_grid": (_INT, [_VP, _INT, _P, _I, _D, _I]),
    "swrt_set_field_psi": (_INT, [_VP, _INT, _P, _I, _D]),
    "swrt_set_field_qk": (_INT, [_VP, _INT, _P, _I, _D, _D, _D, _D, _I]),
    "swrt_set_field_q": (_INT, [_VP, _INT, _P, _I, _D, _D, _D, _D, _I]),
    "swrt_get_field_grid": (_INT, [_VP, _INT, _P]),
    "swrt_get_psi_grid": (_INT, [_VP, _INT, _P]),
    "swrt_field_grid": (_I, [_VP, _INT]),
    "swrt_g2k": (_INT, [_VP, _P, _I, _P]),
    "swrt_k2g": (_INT, [_VP, _P, _I, _P]),
    "swrt_interpolate": (_INT, [_VP, _P, _I, _I, _D, _D, _D, _P, _P, _I, _P]),
    "swrt_eval": (_INT, [_VP, _P, _P, _I, _INT, _D, _D, _P]),
    "swrt_packets_set": (_INT, [_VP, _P, _P, _I]),
    "swrt_packets_get": (_INT, [_VP, _P, _P]),
    "swrt_packets_get_device": (_INT, [_VP, _VP, _VP, ctypes.c_int64]),
    "swrt_packets_count": (_I, [_VP]),
    "swrt_set_locality": (_INT, [_VP, _I, _I]),
    "swrt_set_kernel": (_INT, [_VP, _INT]),
    "swrt_set_gather_mode": (_INT, [_VP, _INT]),
    "swrt_set_sparse_tiles": (_INT, [_VP, _INT]),
    "swrt_set_packet_streams": (_INT, [_VP, _INT]),
    "swrt_advance": (_INT, [_VP, _D, _I, _D, _D, _INT, _D, _D, _D, _I]),
    "swrt_advance_intervals": (_INT, [_VP, _INT, _VP, _I, _D, _D, _D, _D, _D, _I]),
    "swrt_history_frames": (_I, [_VP]),
    "swrt_history_get": (_INT, [_VP, _I, _I, _P, _P]),
    "swrt_history_reset": (_INT, [_VP]),
    "swrt_leapfrog": (_INT, [_VP, _P, _P, _I, _D, _I, _D, _D, _INT, _D, _D, _D, _I, _P, _P]),
    "swrt_xka_set_fields": (_INT, [_VP, _P, _I, _D, _D]),
    "swrt_xka_set_rsw": (_INT, [_VP, _P, _I, _D, _D, _D]),
    "swrt_xka_get_fields": (_INT, [_VP, _P]),
    "swrt_xka_grid": (_I, [_VP]),
    "swrt_xka_step": (_INT, [_VP, _P, _I, _D, _D, _D, _I, _I, _P]),
    "swrt_spectral_set_modes": (_INT, [_VP, _P, _I, _I, _D, _D, _D]),
    "swrt_spectral_eval": (_INT, [_VP, _P, _P, _I, _INT, _P]),
    "swrt_spectral_leapfrog": (_INT, [_VP, _P, _P, _I, _D, _I, _D, _D, _INT]),
    "swrt_omega_histogram": (_INT, [_VP, _D, _D, _P, _I, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(_D)]),
    "swrt_ode23_f1": (_INT, [_VP, _D, _D, _D, _D, _INT, _D, _D, ctypes.POINTER(_D)]),
    "swrt_ode23_attempt": (_INT, [_VP, _D, _D, _D, _D, _D, _D, _INT, _D, _D, ctypes.POINTER(_D)]),
    "swrt_ode23_accept": (_INT, [_VP]),
    "swrt_ode23_run": (_INT, [_VP, _D, _D, _D, _D, _D, _INT, _D, _D, _D, _P, _I, ctypes.POINTER(_I),
                              ctypes.POINTER(_I)]),
    "swrt_ode23_run_hooked": (_INT, [_VP, _D, _D, _D, _D, _D, _INT, _D, _D, _D, _P, _I, ctypes.POINTER(_I),
                                     ctypes.POINTER(_I), _HOOK, _VP]),
    "swrt_ode23_run_sharded": (_INT, [_VP, _D, _D, _D, _D, _D, _INT, _D, _D, _D, _P, _I, ctypes.POINTER(_I),
                                      ctypes.POINTER(_I), _HOOK, _VP, _REDUCE, _VP]),
    "swrt_ode23_chain_next": (_INT, [_VP, _INT, _INT]),
    "swrt_ode23_replay": (_INT, [_D, _D, _D, _D, _INT, _P, _I, _P, _I, ctypes.POINTER(_I), _P, _I,
                                 ctypes.POINTER(_I), ctypes.POINTER(_I)]),
    "swrt_qg_init": (_INT, [_VP, ctypes.POINTER(QGParams), _I, _P]),
    "swrt_qg_step": (_INT, [_VP, _D, _I]),
    "swrt_qg_step_speculative": (_INT, [_VP, _D]),
    "swrt_qg_resolve": (_INT, [_VP, _INT]),
    "swrt_qg_set_stream": (_INT, [_VP, _INT]),
    "swrt_qg_set_fused": (_INT, [_VP, _INT]),
    "swrt_qg_max_speed": (_INT, [_VP, ctypes.POINTER(_D)]),
    "swrt_qg_max_speed_async": (_INT, [_VP]),
    "swrt_qg_max_speed_result": (_INT, [_VP, ctypes.POINTER(_D)]),
    "swrt_qg_get": (_INT, [_VP, _P, ctypes.POINTER(_D), ctypes.POINTER(ctypes.c_int64)]),
    "swrt_qg_get_q": (_INT, [_VP, _P]),
    "swrt_qg_grid": (_I, [_VP, ctypes.POINTER(_INT)]),
    "swrt_qg_snapshot": (_INT, [_VP, _INT, _INT, _INT, _I]),
    "swrt_qg_snapshot_speculative": (_INT, [_VP, _INT, _I]),
    "swrt_qg_export": (_INT, [_VP, _INT, _INT, _VP, _INT, _VP, _D]),
    "swrt_snapshot_qk": (_INT, [_VP, _INT, _VP, _INT, _VP, _I, _D, _D, _D, _D, _I]),
    "swrt_swap_slots": (_INT, [_VP, _INT, _INT]),
    "swrt_field_div_free": (_INT, [_VP, _INT]),
    "swrt_check_arith": (_INT, [_VP, _I, ctypes.c_uint64, ctypes.POINTER(ctypes.c_int64)]),
    "swrt_synchronize": (_INT, [_VP]),
    "swrt_get_stream": (_INT, [_VP, ctypes.POINTER(_VP)]),
    "swrt_set_timing": (_INT, [_VP, _INT]),
    "swrt_kernel_time": (_INT, [_VP, _INT, ctypes.POINTER(_D), ctypes.POINTER(_I)]),
    "swrt_clock_stamp": (_INT, [_VP, _INT]),
    "swrt_clock_ghz": (_INT, [_VP, ctypes.POINTER(_D), ctypes.POINTER(_D)]),
    "swrt_clock_ghz_stamps": (_INT, [ctypes.POINTER(ctypes.c_uint64), _I, _D, ctypes.POINTER(_D),
                                     ctypes.POINTER(_D)]),
    "swrt_debug_set": (_INT, [_VP, _INT, _I]),
    "swrt_debug_get": (_INT, [_VP, _INT, ctypes.POINTER(_I)]),
}

# swrt_debug_set / swrt_debug_get keys (include/swrt.h)
DEBUG_HAZARD_CHECK = 1
DEBUG_SPIN_US = 2
DEBUG_LEGACY_PARK = 3
DEBUG_HAZARD_CHECKS = 4
DEBUG_QG_JFUSE = 5
DEBUG_QG_UPDATE_COLS = 7
DEBUG_SHARE_SKEW = 8
DEBUG_CORRUPT_COUNT = 9
DEBUG_ODE23_CHAINED = 10
DEBUG_ODE23_FIRST_TAKEN = 11
DEBUG_ODE23_GUESSES_TAKEN = 12
DEBUG_ODE23_SPLIT_RUNS = 13
DEBUG_ODE23_FIRST_CHAINED = 14

_lib = None


class SwrtError(RuntimeError):
    pass


def device_code_sha256(path=None):
    """sha256 of the device code embedded in a libswrt build (its ELF
    .hip_fatbin section: every gfx950 kernel, none of the host code).  PMC
    records carry it (tools/pmc_merge.py), so counters collected on one
    build are never divided by the launch time of another (bench.py)."""
    import hashlib
    import struct
    with open(path or LIB_PATH, "rb") as fh:
        b = fh.read()
    if b[:4] != b"\x7fELF" or b[4] != 2 or b[5] != 1:
        raise ValueError("not a little-endian ELF64 file")
    shoff, = struct.unpack_from("<Q", b, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)

    def sec(i):
        name, _, _, _, off, size = struct.unpack_from("<IIQQQQ", b, shoff + i * shentsize)
        return name, off, size
    _, stroff, _ = sec(shstrndx)
    for i in range(shnum):
        name, off, size = sec(i)
        end = b.index(b"\0", stroff + name)
        if b[stroff + name:end] == b".hip_fatbin":
            return hashlib.sha256(b[off:off + size]).hexdigest()
    raise ValueError("no .hip_fatbin section")


def load():
    """dlopen libswrt.so (no HIP call is made by loading)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not found: the HIP extension is not built "
            "(run `python -c 'import __graft_entry__ as g; g.build()'`). "
            "There is no CPU fallback.")
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def _p(a):
    return None if a is None else a.ctypes.data_as(_P)


def _f64(a, order="C"):
    return np.require(np.asarray(a, dtype=np.float64), requirements=[order[0] + "_CONTIGUOUS", "ALIGNED"])


class Context:
    """Owns one swrt_ctx (device buffers + HIP stream) on one GPU."""

    def __init__(self, device: int = 0):
        self._L = load()
        h = _VP()
        rc = self._L.swrt_create(int(device), ctypes.byref(h))
        if rc != SWRT_OK:
            raise SwrtError(f"swrt_create(device={device}) failed: {ERRORS.get(rc, rc)}")
        self._h = h
        self.device = device
        self._ode23_cb = self._ode23_hook = self._ode23_raised = None  # ode23_run's hook callback
        self._ode23_red_cb = self._ode23_reduce = None  # ... and its reduce callback (sharded runs)
        self.timing_every = 1  # swrt_set_timing's setting (the library default)

    def close(self):
        if getattr(self, "_h", None):
            self._L.swrt_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc, what):
        if rc != SWRT_OK:
            msg = self._L.swrt_last_error(self._h)
            raise SwrtError(f"{what}: {ERRORS.get(rc, rc)}: {msg.decode() if msg else ''}")

    # ---- fields ---------------------------------------------------------
    def set_field_grid(self, slot, planes6, nx, L, ny_period=0):
        planes6 = _f64(planes6)
        assert planes6.size == 6 * nx * nx
        self._chk(self._L.swrt_set_field_grid(self._h, slot, _p(planes6), nx, float(L), ny_period),
                  "swrt_set_field_grid")

    def set_field_psi(self, slot, psi_grid, nx, L):
        psi = _f64(np.asarray(psi_grid, dtype=np.float64).ravel(order="F"))
        assert psi.size == nx * nx
        self._chk(self._L.swrt_set_field_psi(self._h, slot, _p(psi), nx, float(L)), "swrt_set_field_psi")

    def set_field_qk(self, slot, qk, nx, L, K_d2, shear=0.0, k_scale=1.0, ny_period=0):
        qk = np.asarray(qk, dtype=np.complex128)
        kmax = nx // 2 - 1
        assert qk.shape == (2 * kmax + 1, kmax + 1), qk.shape
        buf = _f64(np.asfortranarray(qk).ravel(order="F").view(np.float64))
        self._chk(self._L.swrt_set_field_qk(self._h, slot, _p(buf), nx, float(L), float(K_d2),
                                            float(shear), float(k_scale), ny_period),
                  "swrt_set_field_qk")

    def set_field_q(self, slot, q, L, K_d2, shear=0.0, k_scale=1.0, ny_period=0):
        """grid_U(g2k(q)) into `slot` from a gridded PV frame (swrt_set_field_q)."""
        q = np.asarray(q, dtype=np.float64)
        nx = q.shape[0]
        if q.shape != (nx, nx):
            raise ValueError("q must be nx x nx")
        buf = _f64(q.ravel(order="F"))
        self._chk(self._L.swrt_set_field_q(self._h, slot, _p(buf), nx, float(L), float(K_d2), float(shear),
                                           float(k_scale), int(ny_period)), "swrt_set_field_q")

    def field_grid(self, slot):
        """nx of field slot `slot` (swrt_field_grid); raises if unset."""
        nx = int(self._L.swrt_field_grid(self._h, int(slot)))
        if nx < 0:
            raise SwrtError(f"field slot {slot} is not set")
        return nx

    def _slot_nx(self, slot, nx):
        have = self.field_grid(slot)
        if nx is not None and int(nx) != have:
            raise ValueError(f"slot {slot} holds a {have}^2 grid, not {nx}^2")
        return have

    def get_field_grid(self, slot, nx=None):
        nx = self._slot_nx(slot, nx)
        out = np.empty(6 * nx * nx)
        self._chk(self._L.swrt_get_field_grid(self._h, slot, _p(out)), "swrt_get_field_grid")
        return out.reshape(6, nx * nx)

    def field_div_free(self, slot=0):
        """True if slot's v_y is exactly -u_x (the packet kernels then carry
        five stencil sums; results are unchanged)."""
        rc = self._L.swrt_field_div_free(self._h, int(slot))
        if rc < 0:
            self._chk(rc, "swrt_field_div_free")
        return rc == 1

    def get_psi_grid(self, slot, nx=None):
        nx = self._slot_nx(slot, nx)
        out = np.empty(nx * nx)
        self._chk(self._L.swrt_get_psi_grid(self._h, slot, _p(out)), "swrt_get_psi_grid")
        return out.reshape((nx, nx), order="F")

    def g2k(self, fg):
        fg = np.asarray(fg, dtype=np.float64)
        nx = fg.shape[0]
        kmax = nx // 2 - 1
        src = _f64(fg.ravel(order="F"))
        out = np.empty(2 * (2 * kmax + 1) * (kmax + 1))
        self._chk(self._L.swrt_g2k(self._h, _p(src), nx, _p(out)), "swrt_g2k")
        return out.view(np.complex128).reshape((2 * kmax + 1, kmax + 1), order="F")

    def k2g(self, fk):
        fk = np.asarray(fk, dtype=np.complex128)
        nx = fk.shape[0] + 1
        src = _f64(np.asfortranarray(fk).ravel(order="F").view(np.float64))
        out = np.empty(nx * nx)
        self._chk(self._L.swrt_k2g(self._h, _p(src), nx, _p(out)), "swrt_k2g")
        return out.reshape((nx, nx), order="F")

    # ---- evaluation -------------------------------------------------------
    def interpolate(self, x, y, F, dx, dy, bump):
        F = np.asarray(F, dtype=np.float64)
        nx = F.shape[0]
        nyF = int(np.prod(F.shape[1:]))
        Fc = _f64(F.reshape(nx, -1, order="F")[:, :nx].ravel(order="F"))
        x = np.asarray(x, dtype=np.float64)
        shape = x.shape
        xf = _f64(x.ravel())
        yf = _f64(np.asarray(y, dtype=np.float64).ravel())
        out = np.empty(xf.size)
        self._chk(self._L.swrt_interpolate(self._h, _p(Fc), nx, nyF, float(dx), float(dy), float(bump),
                                           _p(xf), _p(yf), xf.size, _p(out)), "swrt_interpolate")
        return out.reshape(shape)

    def eval(self, x, y, nslots=1, alpha=0.0, bump=1e-13):
        xf = _f64(np.asarray(x, dtype=np.float64).ravel())
        yf = _f64(np.asarray(y, dtype=np.float64).ravel())
        out = np.empty((6, xf.size))
        self._chk(self._L.swrt_eval(self._h, _p(xf), _p(yf), xf.size, nslots, float(alpha), float(bump),
                                    _p(out)), "swrt_eval")
        return out

    # ---- packets ---------------------------------------------------------
    def packets_set(self, x, k):
        """x, k: N x 2 arrays (converted to column-major)."""
        x = np.asfortranarray(x, dtype=np.float64)
        k = np.asfortranarray(k, dtype=np.float64)
        assert x.shape == k.shape and x.ndim == 2 and x.shape[1] == 2
        self._chk(self._L.swrt_packets_set(self._h, _p(x), _p(k), x.shape[0]), "swrt_packets_set")

    def packets_get(self):
        n = self._L.swrt_packets_count(self._h)
        x = np.empty((n, 2), order="F")
        k = np.empty((n, 2), order="F")
        self._chk(self._L.swrt_packets_get(self._h, _p(x), _p(k)), "swrt_packets_get")
        return x, k

    def packets_count(self):
        return int(self._L.swrt_packets_count(self._h))

    def packets_get_device(self, x_ptr, k_ptr, ld):
        """swrt_packets_get_device: original-order state into device buffers
        (addresses, N x 2 column-major with leading dimension ld) on the
        packet stream, no host sync."""
        self._chk(self._L.swrt_packets_get_device(self._h, ctypes.c_void_p(int(x_ptr)), ctypes.c_void_p(int(k_ptr)),
                                                  int(ld)), "swrt_packets_get_device")

    def set_locality(self, rebin_every=4, tile=0):
        self._chk(self._L.swrt_set_locality(self._h, int(rebin_every), int(tile)), "swrt_set_locality")

    def set_kernel(self, variant=0):
        self._chk(self._L.swrt_set_kernel(self._h, int(variant)), "swrt_set_kernel")

    def set_gather_mode(self, mode=0):
        """swrt_set_gather_mode: 0 bit-exact mul-then-add stencil sums (default),
        1 fused multiply-add (tolerance parity, fewer VALU instructions)."""
        self._chk(self._L.swrt_set_gather_mode(self._h, int(mode)), "swrt_set_gather_mode")

    def set_sparse_tiles(self, mode=0):
        """swrt_set_sparse_tiles: 0 auto (below SWRT_SPARSE_BELOW packets per tile), 1 never, 2 always; same bits."""
        self._chk(self._L.swrt_set_sparse_tiles(self._h, int(mode)), "swrt_set_sparse_tiles")

    def set_packet_streams(self, streams=2):
        """swrt_set_packet_streams: 2 (default: tile launches split over two streams) or 1; same bits."""
        self._chk(self._L.swrt_set_packet_streams(self._h, int(streams)), "swrt_set_packet_streams")

    def advance(self, dt, nsteps, f, gH, nslots=1, alpha0=0.0, dalpha=0.0, bump=1e-13, save_every=0):
        self._chk(self._L.swrt_advance(self._h, float(dt), int(nsteps), float(f), float(gH), int(nslots),
                                       float(alpha0), float(dalpha), float(bump), int(save_every)),
                  "swrt_advance")

    def advance_intervals(self, dts, nsub, f, gH, alpha0=0.0, dalpha=0.0, bump=1e-13, save_every=0):
        """len(dts) PDE intervals of nsub steps, interval i blending slots i, i+1
        (swrt_advance_intervals)."""
        d = np.ascontiguousarray(dts, dtype=np.float64)
        self._chk(self._L.swrt_advance_intervals(self._h, int(d.size), _p(d), int(nsub), float(f), float(gH),
                                                 float(alpha0), float(dalpha), float(bump), int(save_every)),
                  "swrt_advance_intervals")

    def history(self, first=0, count=None):
        n = self._L.swrt_packets_count(self._h)
        total = self._L.swrt_history_frames(self._h)
        count = total - first if count is None else count
        hx = np.empty((count, 2, n))
        hk = np.empty((count, 2, n))
        self._chk(self._L.swrt_history_get(self._h, first, count, _p(hx), _p(hk)), "swrt_history_get")
        return hx, hk

    def history_reset(self):
        self._chk(self._L.swrt_history_reset(self._h), "swrt_history_reset")

    def leapfrog(self, x, k, dt, nsteps, f, gH, nslots=1, alpha0=0.0, dalpha=0.0, bump=1e-13,
                 save_every=0):
        x = np.array(x, dtype=np.float64, order="F")
        k = np.array(k, dtype=np.float64, order="F")
        n = x.shape[0]
        nfr = nsteps // save_every if save_every else 0
        hx = np.empty((nfr, 2, n)) if nfr else None
        hk = np.empty((nfr, 2, n)) if nfr else None
        self._chk(self._L.swrt_leapfrog(self._h, _p(x), _p(k), n, float(dt), int(nsteps), float(f),
                                        float(gH), int(nslots), float(alpha0), float(dalpha),
                                        float(bump), int(save_every) if nfr else 0, _p(hx), _p(hk)),
                  "swrt_leapfrog")
        return x, k, hx, hk

    # ---- wave action (step_packet_xka) -------------------------------------
    def xka_set_fields(self, U, GradU, H, dx, dy):
        nx = np.asarray(H).shape[0]
        planes = _f64(np.stack([np.asarray(a, dtype=np.float64).ravel(order="F") for a in
                                (U["u"], U["v"], GradU["u_x"], GradU["u_y"], GradU["v_x"], GradU["v_y"], H)]))
        self._chk(self._L.swrt_xka_set_fields(self._h, _p(planes), nx, float(dx), float(dy)),
                  "swrt_xka_set_fields")

    def xka_set_rsw(self, S, f, Cg, L=2 * np.pi):
        """Background from an RSW state S = [u v eta] (nx x nx x 3), built on
        the GPU as ray_trace_sw/raytrace_sw.m:16-52 does."""
        S = np.asarray(S, dtype=np.float64)
        if S.ndim != 3 or S.shape[2] != 3 or S.shape[0] != S.shape[1]:
            raise ValueError("S must be nx x nx x 3")
        st = _f64(np.stack([S[:, :, i].ravel(order="F") for i in range(3)]))
        self._chk(self._L.swrt_xka_set_rsw(self._h, _p(st), S.shape[0], float(f), float(Cg), float(L)),
                  "swrt_xka_set_rsw")

    def xka_get_fields(self):
        """The current background as (U, GradU, H) dicts/planes (nx x nx)."""
        nx = int(self._L.swrt_xka_grid(self._h))
        out = np.empty((7, nx * nx))
        self._chk(self._L.swrt_xka_get_fields(self._h, _p(out)), "swrt_xka_get_fields")
        p = [out[i].reshape((nx, nx), order="F") for i in range(7)]
        return ({"u": p[0], "v": p[1]}, {"u_x": p[2], "u_y": p[3], "v_x": p[4], "v_y": p[5]}, p[6])

    def xka_step(self, state, C0, f, dt, nsteps, save_every=0):
        """state: n x 5 [x y k l a]; returns (new state, history frames n x 5 or None)."""
        st = np.array(state, dtype=np.float64, order="F")
        n = st.shape[0]
        nfr = nsteps // save_every if save_every else 0
        hist = np.empty((nfr, 5, n)) if nfr else None
        self._chk(self._L.swrt_xka_step(self._h, _p(st), n, float(C0), float(f), float(dt), int(nsteps),
                                        int(save_every) if nfr else 0, _p(hist)), "swrt_xka_step")
        return st, (None if hist is None else hist.transpose(0, 2, 1))

    # ---- exact spectral evaluator -----------------------------------------
    def spectral_set_modes(self, C, kx0, ky0, s):
        C = np.asarray(C, dtype=np.complex128)
        nkx, nky = C.shape
        buf = _f64(np.asfortranarray(C).ravel(order="F").view(np.float64))
        self._chk(self._L.swrt_spectral_set_modes(self._h, _p(buf), nkx, nky, float(kx0), float(ky0), float(s)),
                  "swrt_spectral_set_modes")

    def spectral_eval(self, x, y, precision=64):
        xf = _f64(np.asarray(x, dtype=np.float64).ravel())
        yf = _f64(np.asarray(y, dtype=np.float64).ravel())
        out = np.empty((6, xf.size))
        self._chk(self._L.swrt_spectral_eval(self._h, _p(xf), _p(yf), xf.size, int(precision), _p(out)),
                  "swrt_spectral_eval")
        return out

    def spectral_leapfrog(self, x, k, dt, nsteps, f, gH, precision=64):
        x = np.array(x, dtype=np.float64, order="F")
        k = np.array(k, dtype=np.float64, order="F")
        self._chk(self._L.swrt_spectral_leapfrog(self._h, _p(x), _p(k), x.shape[0], float(dt), int(nsteps),
                                                 float(f), float(gH), int(precision)), "swrt_spectral_leapfrog")
        return x, k

    # ---- diagnostics (load_data.m) -----------------------------------------
    def omega_histogram(self, f, Cg, edges, counts=None):
        """Add this frame's omega histcounts to `counts` (int64); returns
        (counts, mean omega)."""
        edges = _f64(np.asarray(edges, dtype=np.float64))
        nb = edges.size - 1
        counts = np.zeros(nb, dtype=np.int64) if counts is None else counts
        assert counts.dtype == np.int64 and counts.size == nb and counts.flags["C_CONTIGUOUS"]
        mean = _D()
        self._chk(self._L.swrt_omega_histogram(self._h, float(f), float(Cg), _p(edges), nb,
                                               counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
                                               ctypes.byref(mean)), "swrt_omega_histogram")
        return counts, mean.value

    # ---- ode23 device stages (swrt_ode23_*) --------------------------------
    def ode23_f1(self, t, tmax, f, Cg, nslots, thr, bump):
        r = _D()
        self._chk(self._L.swrt_ode23_f1(self._h, float(t), float(tmax), float(f), float(Cg), int(nslots),
                                        float(thr), float(bump), ctypes.byref(r)), "swrt_ode23_f1")
        return r.value

    def ode23_attempt(self, t, h, tnew, tmax, f, Cg, nslots, thr, bump):
        r = _D()
        self._chk(self._L.swrt_ode23_attempt(self._h, float(t), float(h), float(tnew), float(tmax), float(f),
                                             float(Cg), int(nslots), float(thr), float(bump), ctypes.byref(r)),
                  "swrt_ode23_attempt")
        return r.value

    def ode23_accept(self):
        self._chk(self._L.swrt_ode23_accept(self._h), "swrt_ode23_accept")

    def ode23_run(self, t0, tfinal, tmax, f, Cg, nslots, rtol, atol, bump, ts_cap=10_000, hook=None, reduce=None):
        """swrt_ode23_run: the whole ode23 call with the controller in the
        library.  Returns (accepted times, {steps, failed, attempts,
        accepted}); `accepted` counts every accepted time, and a warning is
        raised when more than ts_cap were accepted (the list then holds the
        first ts_cap only).  ``hook``: a callable run once after the first
        launches are queued (swrt_ode23_run_hooked; QG calls only, never the
        packets).  ``reduce``: a callable float -> float, the max over the
        ranks of a sharded run (swrt_ode23_run_sharded; called once for stage
        1 and once per attempt, the same order on every rank).  An exception
        either raises is re-raised after the call."""
        ts = np.empty(ts_cap)
        nts = _I()
        st = (_I * 3)()
        args = (self._h, float(t0), float(tfinal), float(tmax), float(f), float(Cg), int(nslots), float(rtol),
                float(atol), float(bump), _p(ts), int(ts_cap), ctypes.byref(nts), st)
        if hook is None and reduce is None:
            self._chk(self._L.swrt_ode23_run(*args), "swrt_ode23_run")
        else:
            # one ctypes callback per context (made once), calling this call's hook
            if self._ode23_cb is None:
                def _call(_user):
                    h, self._ode23_hook = self._ode23_hook, None
                    try:
                        if h is not None:
                            h()
                    except BaseException as e:  # ctypes would print and drop it
                        self._ode23_raised = e
                self._ode23_cb = _HOOK(_call)
            self._ode23_hook, self._ode23_raised = hook, None
            if reduce is None:
                rc = self._L.swrt_ode23_run_hooked(*args, self._ode23_cb if hook is not None else _HOOK(), None)
                name = "swrt_ode23_run_hooked"
            else:
                if self._ode23_red_cb is None:
                    def _red(vp, _user):
                        try:
                            vp[0] = float(self._ode23_reduce(vp[0]))
                            return 0
                        except BaseException as e:
                            if self._ode23_raised is None:
                                self._ode23_raised = e
                            return 1
                    self._ode23_red_cb = _REDUCE(_red)
                self._ode23_reduce = reduce
                rc = self._L.swrt_ode23_run_sharded(*args, self._ode23_cb if hook is not None else _HOOK(), None,
                                                    self._ode23_red_cb, None)
                self._ode23_reduce = None
                name = "swrt_ode23_run_sharded"
            self._ode23_hook = None
            raised, self._ode23_raised = self._ode23_raised, None
            if raised is not None:
                raise raised
            self._chk(rc, name)
        # ts_cap bounds the recorded times only (the interval always completes)
        if nts.value > ts_cap:
            import warnings
            warnings.warn(f"swrt_ode23_run accepted {nts.value} times; only the first ts_cap={ts_cap} are returned",
                          RuntimeWarning, stacklevel=2)
        return ts[:min(nts.value, ts_cap)].copy(), {"steps": st[0], "failed": st[1], "attempts": st[2],
                                                    "accepted": nts.value}

    def ode23_chain_next(self, slot_a, slot_b):
        """swrt_ode23_chain_next: the running (or next) ode23_run queues the
        next call's stage 1 with slots (slot_a, slot_b) as its slots 0 / 1
        when it ends; the next call takes it only if it computes the same."""
        self._chk(self._L.swrt_ode23_chain_next(self._h, int(slot_a), int(slot_b)), "swrt_ode23_chain_next")

    # ---- owner-driver hand-off (swrt_qg_export / swrt_snapshot_qk) -----------
    def qg_export(self, dst, which=0, layer=0, stream=None, tail=0.0, fenced=False):
        """Layer `layer` of the current (0) / previous (1) qk in the device's
        half-plane order (ky fastest), then `tail`, into `dst`: a float64
        numpy array of 2*(2kmax+1)*(kmax+1) + 1 values (host copy, returns
        when done), or an int device address (queued; ordered after and
        before the work of the hipStream_t `stream`, default the packet
        stream — ``fenced``: only before it, the caller guarantees dst is
        free; swrt_qg_export dst_mode 2)."""
        if isinstance(dst, np.ndarray):
            if dst.dtype != np.float64 or not dst.flags["C_CONTIGUOUS"] or dst.size != 2 * self._qg_nhalf() + 1:
                raise ValueError("dst must be a contiguous float64 array of 2*(2kmax+1)*(kmax+1) + 1 values")
            self._chk(self._L.swrt_qg_export(self._h, int(which), int(layer), dst.ctypes.data_as(_VP), 0, None,
                                             float(tail)), "swrt_qg_export")
        else:
            self._chk(self._L.swrt_qg_export(self._h, int(which), int(layer), _VP(int(dst)), 2 if fenced else 1,
                                             None if stream is None else _VP(int(stream)), float(tail)),
                      "swrt_qg_export")

    def _qg_nhalf(self):
        kmax = self._qg_nx // 2 - 1
        return (2 * kmax + 1) * (kmax + 1)

    def snapshot_qk(self, slot, qk, nx, L, K_d2, shear=0.0, k_scale=1.0, ny_period=0, stream=None):
        """grid_U of a half plane in qg_export's order into `slot`
        (swrt_snapshot_qk): `qk` a float64 numpy array (host) or an int device
        address (read after / before `stream`'s work)."""
        kmax = int(nx) // 2 - 1
        nh = (2 * kmax + 1) * (kmax + 1)
        if isinstance(qk, np.ndarray):
            if qk.dtype != np.float64 or not qk.flags["C_CONTIGUOUS"] or qk.size != 2 * nh:
                raise ValueError("qk must be a contiguous float64 array of 2*(2kmax+1)*(kmax+1) values")
            src, on_dev, st = qk.ctypes.data_as(_VP), 0, None
        else:
            src, on_dev, st = _VP(int(qk)), 1, None if stream is None else _VP(int(stream))
        self._chk(self._L.swrt_snapshot_qk(self._h, int(slot), src, on_dev, st, int(nx), float(L), float(K_d2),
                                           float(shear), float(k_scale), int(ny_period)), "swrt_snapshot_qk")

    # ---- QG PDE stepper (swrt_qg_*) ---------------------------------------
    def qg_init(self, params: QGParams, nx, qk):
        """qk: (2kmax+1, kmax+1) complex, or (2kmax+1, kmax+1, nlayers)."""
        qk = np.asarray(qk, dtype=np.complex128)
        if qk.ndim == 2:
            qk = qk[:, :, None]
        kmax = nx // 2 - 1
        assert qk.shape == (2 * kmax + 1, kmax + 1, params.nlayers), qk.shape
        buf = _f64(np.asfortranarray(qk).ravel(order="F").view(np.float64))
        self._qg_shape = (2 * kmax + 1, kmax + 1, params.nlayers)
        self._qg_nx = nx
        self._chk(self._L.swrt_qg_init(self._h, ctypes.byref(params), nx, _p(buf)), "swrt_qg_init")

    def qg_step(self, dt, nsteps=1):
        self._chk(self._L.swrt_qg_step(self._h, float(dt), int(nsteps)), "swrt_qg_step")

    def qg_step_speculative(self, dt):
        """swrt_qg_step_speculative: the next step with dt, its transforms and CFL read-back queued into
        spare buffers; the committed state is kept until qg_resolve."""
        self._chk(self._L.swrt_qg_step_speculative(self._h, float(dt)), "swrt_qg_step_speculative")

    def qg_resolve(self, accept):
        """swrt_qg_resolve: accept (the speculative step becomes current) or drop it."""
        self._chk(self._L.swrt_qg_resolve(self._h, int(bool(accept))), "swrt_qg_resolve")

    def qg_set_stream(self, separate=True):
        """QG PDE on its own stream, overlapping the packet launches (swrt_qg_set_stream)."""
        self._chk(self._L.swrt_qg_set_stream(self._h, int(bool(separate))), "swrt_qg_set_stream")

    def qg_set_fused(self, on=True):
        """One batched transform per qk for the step, CFL speed and snapshot (swrt_qg_set_fused)."""
        self._chk(self._L.swrt_qg_set_fused(self._h, int(bool(on))), "swrt_qg_set_fused")
        self.qg_fused = bool(on)

    def qg_max_speed(self):
        u = _D()
        self._chk(self._L.swrt_qg_max_speed(self._h, ctypes.byref(u)), "swrt_qg_max_speed")
        return u.value

    def qg_max_speed_async(self):
        self._chk(self._L.swrt_qg_max_speed_async(self._h), "swrt_qg_max_speed_async")

    def qg_max_speed_result(self):
        u = _D()
        self._chk(self._L.swrt_qg_max_speed_result(self._h, ctypes.byref(u)), "swrt_qg_max_speed_result")
        return u.value

    def qg_get(self):
        """-> (qk (2kmax+1, kmax+1, nlayers) complex, t, steps)."""
        out = np.empty(2 * int(np.prod(self._qg_shape)))
        t = _D()
        s = ctypes.c_int64()
        self._chk(self._L.swrt_qg_get(self._h, _p(out), ctypes.byref(t), ctypes.byref(s)), "swrt_qg_get")
        qk = out.view(np.complex128).reshape(self._qg_shape, order="F")
        return qk, t.value, s.value

    def qg_get_q(self):
        """-> q grid (nx, nx, nlayers), column-major per layer (k2g of each layer)."""
        nx, nl = self._qg_nx, self._qg_shape[2]
        out = np.empty(nx * nx * nl)
        self._chk(self._L.swrt_qg_get_q(self._h, _p(out)), "swrt_qg_get_q")
        return out.reshape((nx, nx, nl), order="F")

    def qg_snapshot(self, slot, which=0, layer=0, ny_period=0):
        self._chk(self._L.swrt_qg_snapshot(self._h, int(slot), int(which), int(layer), int(ny_period)),
                  "swrt_qg_snapshot")

    def qg_snapshot_speculative(self, slot, ny_period=0):
        """swrt_qg_snapshot_speculative: layer 0's grid_U of the pending
        speculative step into `slot` (what qg_snapshot(slot) writes after
        accepting it)."""
        self._chk(self._L.swrt_qg_snapshot_speculative(self._h, int(slot), int(ny_period)),
                  "swrt_qg_snapshot_speculative")

    def swap_slots(self, a=0, b=1):
        self._chk(self._L.swrt_swap_slots(self._h, int(a), int(b)), "swrt_swap_slots")

    # ---- runtime ---------------------------------------------------------
    def synchronize(self):
        self._chk(self._L.swrt_synchronize(self._h), "swrt_synchronize")

    def check_arith(self, n=1 << 20, seed=1):
        """Bit-exactness of the hot loop's short sqrt / reciprocal / drift
        sequences against the device's IEEE operations over 16*n random
        operands (swrt_check_arith): mismatch counts (sqrt, 1/w, drift)."""
        out = (ctypes.c_int64 * 3)()
        self._chk(self._L.swrt_check_arith(self._h, int(n), int(seed), out), "swrt_check_arith")
        return tuple(out)

    def stream(self):
        s = _VP()
        self._chk(self._L.swrt_get_stream(self._h, ctypes.byref(s)), "swrt_get_stream")
        return s.value

    def set_timing(self, every=1):
        self._chk(self._L.swrt_set_timing(self._h, int(every)), "swrt_set_timing")
        self.timing_every = int(every)

    def kernel_time(self, reset=True):
        ms = _D()
        n = _I()
        self._chk(self._L.swrt_kernel_time(self._h, int(reset), ctypes.byref(ms), ctypes.byref(n)),
                  "swrt_kernel_time")
        return ms.value, n.value

    def clock_stamp(self, which):
        """swrt_clock_stamp: 0 before, 1 after a region of packet-stream work."""
        self._chk(self._L.swrt_clock_stamp(self._h, int(which)), "swrt_clock_stamp")

    def clock_ghz(self):
        """swrt_clock_ghz: (median observed shader clock in GHz, relative spread) between the stamps."""
        g, s = _D(), _D()
        self._chk(self._L.swrt_clock_ghz(self._h, ctypes.byref(g), ctypes.byref(s)), "swrt_clock_ghz")
        return g.value, s.value

    def debug_set(self, key, value):
        """swrt_debug_set: DEBUG_HAZARD_CHECK, DEBUG_SPIN_US, DEBUG_LEGACY_PARK (test infrastructure)."""
        self._chk(self._L.swrt_debug_set(self._h, int(key), int(value)), "swrt_debug_set")

    def debug_get(self, key):
        v = _I()
        self._chk(self._L.swrt_debug_get(self._h, int(key), ctypes.byref(v)), "swrt_debug_get")
        return v.value


def ode23_replay(t0, tfinal, raw, rtol=1e-3, atol=1e-6, dev_first=True, ts_cap=100_000):
    """swrt_ode23_replay: the library's ode23 controller (swrt_ode23_ctl.cpp)
    over a scripted raw-error sequence, on the host (no GPU, no context).
    raw[0] = stage 1's max, then one per attempt the controller consumes.
    Returns (status, attempts (n, 4) [t, h, tnew, raw], accepted times, stats
    dict); status is SWRT_OK, "below hmin" or "script exhausted"."""
    L = load()
    raw = np.ascontiguousarray(raw, dtype=np.float64)
    cap = max(1, raw.size)
    log = np.empty(4 * cap)
    ts = np.empty(ts_cap)
    nlog, nts = _I(), _I()
    st = (_I * 9)()
    rc = L.swrt_ode23_replay(float(t0), float(tfinal), float(rtol), float(atol), int(bool(dev_first)), _p(raw),
                             raw.size, _p(log), cap, ctypes.byref(nlog), _p(ts), ts_cap, ctypes.byref(nts), st)
    status = {SWRT_OK: SWRT_OK, 3: "below hmin", 1: "script exhausted"}.get(rc, rc)
    keys = ("steps", "failed", "attempts", "first_taken", "guesses", "taken_maxstep", "taken_ramp_maxstep",
            "taken_ramp_5x", "gate_violations")
    return (status, log[:4 * min(nlog.value, cap)].reshape(-1, 4).copy(), ts[:min(nts.value, ts_cap)].copy(),
            {k: int(v) for k, v in zip(keys, st)})


def clock_ghz_stamps(stamps, realtime_hz=100e6):
    """swrt_clock_ghz_stamps: (GHz, spread) from probe stamps shaped (2, waves,
    3) = start/end x wave x {cycles, realtime ticks, CU id}; raises SwrtError
    when no CU holds both a start and an end wave (host only)."""
    L = load()
    a = np.ascontiguousarray(stamps, dtype=np.uint64)
    if a.ndim != 3 or a.shape[0] != 2 or a.shape[2] != 3:
        raise ValueError("stamps must be (2, waves, 3)")
    g, s = _D(), _D()
    rc = L.swrt_clock_ghz_stamps(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64)), a.shape[1], float(realtime_hz),
                                 ctypes.byref(g), ctypes.byref(s))
    if rc != SWRT_OK:
        raise SwrtError(f"swrt_clock_ghz_stamps: {ERRORS.get(rc, rc)}: no CU with both a start and an end stamp"
                        if rc == 3 else f"swrt_clock_ghz_stamps: {ERRORS.get(rc, rc)}")
    return g.value, s.value


def exported_symbols():
    """Names the header declares (for the ABI export test)."""
    return list(SIGNATURES)


if __name__ == "__main__":  # pragma: no cover
    load()
    print("libswrt loaded:", LIB_PATH, file=sys.stderr)
