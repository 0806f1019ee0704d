"""ipo_amd -- Python host mirror of the ipo-hip C ABI (include/ipo_hip.h).

The product is the C-ABI shared library ``lib/libipo_hip.so`` (HIP kernels for
gfx950 + native host code).  This module is a thin ctypes binding used by the
tests and ``bench.py``; it mirrors the reference's operator interface:

* :func:`solver`          -- ``solver()`` of src/common/solve.c:24-26 (hsd.c / intpt.c)
* :class:`Ldlt`           -- ``ldltfac()`` / ``forwardbackward()`` of src/ipo/ldlt.h
* :func:`run_mps`         -- the ``ipo file.mps`` driver (src/common/main.c:16-58)

There is no CPU fallback: if the library is missing or no GPU is present the
calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
import tempfile
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_PATH = os.path.join(PKG_ROOT, "lib", "libipo_hip.so")

STATUS_TEXT = {
    0: "optimal solution", 1: "primal unbounded", 2: "primal infeasible", 3: "dual unbounded",
    4: "dual infeasible", 5: "iteration limit", 6: "infinite lower bounds - not implemented",
    7: "suboptimal solution",
}
METHODS = {"hsd": 0, "intpt": 1, "hsdls": 2}


class IpoHipError(RuntimeError):
    pass


class Stats(C.Structure):
    _fields_ = [
        ("iters", C.c_int), ("status", C.c_int),
        ("t_setup_s", C.c_double), ("t_solve_s", C.c_double),
        ("factor_ms", C.c_double), ("solve_ms", C.c_double),
        ("factors", C.c_long), ("solves", C.c_long), ("rawsolves", C.c_long), ("refine_passes", C.c_long),
        ("final_mu", C.c_double), ("final_pobj", C.c_double), ("final_dobj", C.c_double),
        ("final_pinf", C.c_double), ("final_dinf", C.c_double),
        ("lnz", C.c_long), ("narth", C.c_double), ("nsup", C.c_int), ("nlevels", C.c_int),
        ("flops_factor", C.c_double), ("lx_bytes", C.c_double),
        ("update_ms", C.c_double), ("panel_ms", C.c_double), ("sweep_ms", C.c_double),
        ("update_launches", C.c_long), ("panel_launches", C.c_long),
        ("flops_update", C.c_double), ("bytes_update", C.c_double),
        ("phase_ms", C.c_double * 8), ("phase_launches", C.c_long * 8), ("phase_count", C.c_long * 8),
        ("phase_flops", C.c_double * 8), ("phase_bytes", C.c_double * 8),
        ("tail_repairs", C.c_long), ("tail_dep_rounds", C.c_long), ("tail_chain_aborts", C.c_long),
    ]

    def as_dict(self) -> dict:
        d = {}
        for k, _ in self._fields_:
            v = getattr(self, k)
            d[k] = list(v) if isinstance(v, C.Array) else v
        return d


_lib = None
_libc = None

PHASES = ["gather", "diag", "trsm", "tail_syrk", "forward", "backward", "tail", "unused"]

EXPORTED = [
    "solver", "ldltfac", "forwardbackward", "inv_clo",
    "ipo_hip_solve", "ipo_hip_run_mps", "ipo_hip_run_mps_ex", "ipo_hip_mps_dims", "ipo_hip_mps_load",
    "ipo_hip_mps_load_ex", "ipo_hip_write_sol",
    "ipo_hip_kkt_create", "ipo_hip_kkt_destroy", "ipo_hip_kkt_factor", "ipo_hip_kkt_solve",
    "ipo_hip_kkt_info", "ipo_hip_kkt_perm", "ipo_hip_kkt_pivots", "ipo_hip_symbolic",
    "ipo_hip_device_count", "ipo_hip_device_synchronize", "ipo_hip_last_error", "ipo_hip_version",
    "ipo_hip_ctx_create", "ipo_hip_ctx_run", "ipo_hip_ctx_download", "ipo_hip_ctx_destroy",
    "ipo_hip_ctx_setup_seconds", "ipo_hip_kkt_set_epsdiag",
    "ipo_hip_synth_random", "ipo_hip_synth_block_angular", "ipo_hip_symbolic_forced",
    "ipo_hip_set_device", "ipo_hip_rccl_unique_id", "ipo_hip_ctx_create_shard", "ipo_hip_vector_bench",
    "ipo_hip_dot_ordered",
    "ipo_hip_kkt_create_q", "ipo_hip_ldlt_set_q", "ipo_hip_symbolic_q", "ipo_hip_mps_quads",
]

# int (*)(void *user, double *buf, long n, int op)  -- ipo_hip_allreduce_fn
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.POINTER(C.c_double), C.c_long, C.c_int)

_P = C.c_void_p
_I = C.c_int
_D = C.c_double


def lib() -> C.CDLL:
    """Load libipo_hip.so (raises if it was not built)."""
    global _lib, _libc
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise IpoHipError(f"{LIB_PATH} missing: run `make -C linear-programming-vanderbei_amd` "
                          "(or __graft_entry__.build())")
    L = C.CDLL(LIB_PATH)
    L.solver.argtypes = [_I, _I, _I, _P, _P, _P, _P, _P, _D, _P, _P, _P, _P]
    L.solver.restype = _I
    L.ldltfac.argtypes = [_I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _I]
    L.ldltfac.restype = None
    L.forwardbackward.argtypes = [_P, _P, _P, _P]
    L.forwardbackward.restype = None
    L.inv_clo.argtypes = []
    L.inv_clo.restype = None
    L.ipo_hip_solve.argtypes = [_I, _I, _I, _I, _P, _P, _P, _P, _P, _D, _P, _P, _P, _P, _P, _I, _I, C.POINTER(Stats)]
    L.ipo_hip_solve.restype = _I
    L.ipo_hip_run_mps.argtypes = [C.c_char_p, _I, _P, _I, C.POINTER(Stats)]
    L.ipo_hip_run_mps.restype = _I
    L.ipo_hip_run_mps_ex.argtypes = [C.c_char_p, _I, _I, C.c_char_p, _P, _I, C.POINTER(Stats)]
    L.ipo_hip_run_mps_ex.restype = _I
    L.ipo_hip_mps_load_ex.argtypes = [C.c_char_p, _I, C.POINTER(_I), C.POINTER(_I), C.POINTER(_I), _P, _P, _P, _P, _P,
                                      C.POINTER(_D)]
    L.ipo_hip_mps_load_ex.restype = _I
    L.ipo_hip_write_sol.argtypes = [C.c_char_p, _I, _P, _P, _P, C.c_char_p]
    L.ipo_hip_write_sol.restype = _I
    L.ipo_hip_mps_dims.argtypes = [C.c_char_p] + [C.POINTER(_I)] * 6
    L.ipo_hip_mps_dims.restype = _I
    L.ipo_hip_mps_load.argtypes = [C.c_char_p, C.POINTER(_I), C.POINTER(_I), C.POINTER(_I), _P, _P, _P, _P, _P,
                                   C.POINTER(_D)]
    L.ipo_hip_mps_load.restype = _I
    L.ipo_hip_kkt_create.argtypes = [_I, _I, _P, _P, _P]
    L.ipo_hip_kkt_create.restype = _P
    L.ipo_hip_kkt_create_q.argtypes = [_I, _I, _P, _P, _P, _P, _P, _P, _I]
    L.ipo_hip_kkt_create_q.restype = _P
    L.ipo_hip_ldlt_set_q.argtypes = [_I, _P, _P, _P, _I]
    L.ipo_hip_ldlt_set_q.restype = _I
    L.ipo_hip_symbolic_q.argtypes = [_I, _I, _P, _P, _P, _P, _P, C.POINTER(C.c_long), C.POINTER(_D), C.POINTER(_I),
                                     C.POINTER(_I), C.POINTER(_I), C.POINTER(_I)]
    L.ipo_hip_symbolic_q.restype = _I
    L.ipo_hip_mps_quads.argtypes = [C.c_char_p, _P, _P, _P, _P, _P]
    L.ipo_hip_mps_quads.restype = _I
    L.ipo_hip_kkt_destroy.argtypes = [_P]
    L.ipo_hip_kkt_destroy.restype = None
    L.ipo_hip_kkt_factor.argtypes = [_P, _P, _P]
    L.ipo_hip_kkt_factor.restype = _I
    L.ipo_hip_kkt_solve.argtypes = [_P, _P, _P, _P, _P]
    L.ipo_hip_kkt_solve.restype = _I
    L.ipo_hip_kkt_info.argtypes = [_P, C.POINTER(C.c_long), C.POINTER(_D), C.POINTER(_I), C.POINTER(_I),
                                   C.POINTER(_I), C.POINTER(_I), C.POINTER(_D), C.POINTER(_I), C.POINTER(_I)]
    L.ipo_hip_kkt_info.restype = _I
    L.ipo_hip_kkt_perm.argtypes = [_P, _P]
    L.ipo_hip_kkt_perm.restype = _I
    L.ipo_hip_kkt_pivots.argtypes = [_P, _P, _P]
    L.ipo_hip_kkt_pivots.restype = _I
    L.ipo_hip_kkt_set_epsdiag.argtypes = [_P, _D]
    L.ipo_hip_kkt_set_epsdiag.restype = None
    L.ipo_hip_symbolic.argtypes = [_I, _I, _P, _P, _P, C.POINTER(C.c_long), C.POINTER(_D), C.POINTER(_I),
                                   C.POINTER(_I), C.POINTER(_I), C.POINTER(_I)]
    L.ipo_hip_symbolic.restype = _I
    L.ipo_hip_ctx_create.argtypes = [_I, _I, _P, _P, _P, _P, _P, _D]
    L.ipo_hip_ctx_create.restype = _P
    L.ipo_hip_ctx_run.argtypes = [_P, _I, _I, _P, _I, C.POINTER(Stats)]
    L.ipo_hip_ctx_run.restype = _I
    L.ipo_hip_ctx_download.argtypes = [_P, _P, _P, _P, _P]
    L.ipo_hip_ctx_download.restype = None
    L.ipo_hip_ctx_destroy.argtypes = [_P]
    L.ipo_hip_ctx_destroy.restype = None
    L.ipo_hip_ctx_setup_seconds.argtypes = [_P]
    L.ipo_hip_ctx_setup_seconds.restype = _D
    L.ipo_hip_dot_ordered.argtypes = [_P, _P, _I, _P]
    L.ipo_hip_dot_ordered.restype = _I
    L.ipo_hip_vector_bench.argtypes = [_I, _I, _P, _P, _P, _I, _P, _P]
    L.ipo_hip_vector_bench.restype = _I
    L.ipo_hip_synth_random.argtypes = [_I, _I, _I, _I, C.c_ulonglong, C.POINTER(_I)] + [_P] * 9
    L.ipo_hip_synth_random.restype = _I
    L.ipo_hip_synth_block_angular.argtypes = [_I] * 7 + [C.c_ulonglong] + [C.POINTER(_I)] * 3 + [_P] * 9
    L.ipo_hip_synth_block_angular.restype = _I
    L.ipo_hip_symbolic_forced.argtypes = [_I, _I, _P, _P, _I, _P, _P, C.POINTER(C.c_long), C.POINTER(_I),
                                          C.POINTER(_I), C.POINTER(_I)]
    L.ipo_hip_symbolic_forced.restype = _I
    L.ipo_hip_set_device.argtypes = [_I]
    L.ipo_hip_set_device.restype = _I
    L.ipo_hip_rccl_unique_id.argtypes = [_P]
    L.ipo_hip_rccl_unique_id.restype = _I
    L.ipo_hip_ctx_create_shard.argtypes = [_I, _I, _P, _P, _P, _P, _P, _D, _I, _I, _I, C.c_long, _I, _I, _P, _P, _P]
    L.ipo_hip_ctx_create_shard.restype = _P
    L.ipo_hip_device_count.restype = _I
    L.ipo_hip_device_synchronize.restype = _I
    L.ipo_hip_last_error.restype = C.c_char_p
    L.ipo_hip_version.restype = C.c_char_p
    _lib = L
    _libc = C.CDLL(None)
    _libc.fopen.restype = _P
    _libc.fopen.argtypes = [C.c_char_p, C.c_char_p]
    _libc.fclose.argtypes = [_P]
    _libc.fflush.argtypes = [_P]
    return L


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def last_error() -> str:
    return lib().ipo_hip_last_error().decode()


def device_count() -> int:
    return lib().ipo_hip_device_count()


def device_synchronize() -> None:
    """Wait for every stream of this process's device (hipDeviceSynchronize)."""
    if lib().ipo_hip_device_synchronize():
        raise IpoHipError("device_synchronize: " + last_error())


def require_gpu() -> None:
    if device_count() < 1:
        raise IpoHipError("no HIP device visible: ipo-hip has no CPU fallback")


# ----------------------------------------------------------------- MPS front end
@dataclass
class SolverForm:
    """Problem in the form solver() takes: max c'x + f, Ax <= b, x >= 0 (A CSC)."""
    m: int
    n: int
    kA: np.ndarray
    iA: np.ndarray
    A: np.ndarray
    b: np.ndarray
    c: np.ndarray
    f: float

    @property
    def nz(self) -> int:
        return int(self.kA[-1])

    def transpose(self):
        """CSR of A (= CSC of A'), stable like linalg.c:75-103."""
        counts = np.bincount(self.iA, minlength=self.m)
        kAt = np.zeros(self.m + 1, np.int32)
        np.cumsum(counts, out=kAt[1:])
        cols = np.repeat(np.arange(self.n, dtype=np.int32), np.diff(self.kA))
        order = np.argsort(self.iA, kind="stable")
        return kAt, cols[order].astype(np.int32), self.A[order].copy()


def mps_dims(path: str):
    """(m0, n0, nz0, m, n, nz, status) of an MPS file (solve.c:62 and hsd.c:117 lines)."""
    v = [C.c_int(0) for _ in range(6)]
    st = lib().ipo_hip_mps_dims(path.encode(), *[C.byref(x) for x in v])
    return tuple(x.value for x in v) + (st,)


SPLIT_FREE = 1      # include/ipo_hip.h IPO_HIP_SPLIT_FREE


def mps_quads(path: str):
    """The QUADS section as the reference's reader keeps it (symmetric n x n
    CSC over the file's columns): (kQ, iQ, Q), or None without QUADS."""
    L = lib()
    b = path.encode()
    n, qnz = C.c_int(), C.c_int()
    rc = L.ipo_hip_mps_quads(b, C.byref(n), C.byref(qnz), None, None, None)
    if rc:
        raise IpoHipError(f"mps_quads: error {rc}: " + last_error())
    if qnz.value < 0:
        return None
    kQ = np.zeros(n.value + 1, np.int32)
    iQ = np.zeros(max(qnz.value, 1), np.int32)
    Q = np.zeros(max(qnz.value, 1), np.float64)
    L.ipo_hip_mps_quads(b, None, None, _ptr(kQ), _ptr(iQ), _ptr(Q))
    return kQ, iQ[:qnz.value], Q[:qnz.value]


def load_mps(path: str, free: str = "abort") -> SolverForm:
    """Read + normalise an MPS file with the native front end (lp_io.cpp).
    free="split": the free-variable extension (split / reflected columns)
    instead of the reference's abort (status 3)."""
    L = lib()
    fl = SPLIT_FREE if free == "split" else 0
    m, n, nz = C.c_int(0), C.c_int(0), C.c_int(0)
    st = L.ipo_hip_mps_load_ex(path.encode(), fl, C.byref(m), C.byref(n), C.byref(nz), None, None, None, None, None,
                               None)
    if st:
        raise IpoHipError(f"mps load {path}: status {st} {last_error()}")
    kA = np.zeros(n.value + 1, np.int32)
    iA = np.zeros(nz.value, np.int32)
    A = np.zeros(nz.value, np.float64)
    b = np.zeros(m.value, np.float64)
    c = np.zeros(n.value, np.float64)
    f = C.c_double(0.0)
    L.ipo_hip_mps_load_ex(path.encode(), fl, C.byref(m), C.byref(n), C.byref(nz), _ptr(kA), _ptr(iA), _ptr(A), _ptr(b),
                          _ptr(c), C.byref(f))
    return SolverForm(m.value, n.value, kA, iA, A, b, c, f.value)


def write_sol(path: str, x, y, z, solfile: str, free: str = "abort") -> None:
    """writesol (iolp.c:976-1045) of MPS file `path` from solver()-form
    vectors of its normalisation (host code)."""
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    z = np.ascontiguousarray(z, np.float64)
    if lib().ipo_hip_write_sol(path.encode(), SPLIT_FREE if free == "split" else 0, _ptr(x), _ptr(y), _ptr(z),
                               solfile.encode()):
        raise IpoHipError("write_sol: " + last_error())


def _capture(fn):
    """Run fn(FILE*) and return (result, text written)."""
    lib()
    fd, path = tempfile.mkstemp(prefix="ipo_hip_", suffix=".txt")
    os.close(fd)
    fp = _libc.fopen(path.encode(), b"w")
    try:
        r = fn(fp)
    finally:
        _libc.fflush(fp)
        _libc.fclose(fp)
    with open(path) as fh:
        text = fh.read()
    os.unlink(path)
    return r, text


def run_mps(path: str, method: str = "hsd", timing: bool = False, free: str = "abort", solfile: str = None):
    """Equivalent of `ipo path` (main.c) on the GPU.  Returns (status, stdout text, stats dict).
    free="split": the free-variable extension; solfile: write the writesol report there."""
    require_gpu()
    st = Stats()
    fl = SPLIT_FREE if free == "split" else 0
    status, text = _capture(lambda fp: lib().ipo_hip_run_mps_ex(path.encode(), METHODS[method], fl,
                                                               solfile.encode() if solfile else None, fp, int(timing),
                                                               C.byref(st)))
    return status, text, st.as_dict()


def solver(p: SolverForm, method: str = "hsd", trace: bool = False, max_iter: int = 200, timing: bool = False):
    """solver() on host arrays.  Returns dict(status, x, y, w, z, stats, trace)."""
    require_gpu()
    x = np.zeros(p.n, np.float64)
    z = np.zeros(p.n, np.float64)
    y = np.zeros(p.m, np.float64)
    w = np.zeros(p.m, np.float64)
    st = Stats()
    kA = np.ascontiguousarray(p.kA, np.int32)
    iA = np.ascontiguousarray(p.iA, np.int32)
    A = np.ascontiguousarray(p.A, np.float64)
    b = np.ascontiguousarray(p.b, np.float64)
    c = np.ascontiguousarray(p.c, np.float64)

    def call(fp):
        return lib().ipo_hip_solve(METHODS[method], p.m, p.n, p.nz, _ptr(iA), _ptr(kA), _ptr(A), _ptr(b), _ptr(c),
                                   float(p.f), _ptr(x), _ptr(y), _ptr(w), _ptr(z), fp, max_iter, int(timing),
                                   C.byref(st))
    if trace:
        status, text = _capture(call)
    else:
        status, text = call(None), ""
    return {"status": status, "x": x, "y": y, "w": w, "z": z, "stats": st.as_dict(), "trace": text}


# ----------------------------------------------------------------- KKT factor
class KktFactor:
    """Device LDL' of K = [-E A; A' D] for the solver's A (m x n CSC)."""

    def __init__(self, m, n, kA, iA, A, q=None, qmax=1):
        """q = (kQ, iQ, Q): a Q block on the y-nodes, K_yy = -max(E, eps) -
        qmax Q (ldlt.c:253-256; Q m x m, full symmetric CSC)."""
        require_gpu()
        self.m, self.n = m, n
        self._keep = [np.ascontiguousarray(kA, np.int32), np.ascontiguousarray(iA, np.int32),
                      np.ascontiguousarray(A, np.float64)]
        if q is None:
            self.h = lib().ipo_hip_kkt_create(m, n, *[_ptr(a) for a in self._keep])
        else:
            self._keep += [np.ascontiguousarray(q[0], np.int32), np.ascontiguousarray(q[1], np.int32),
                           np.ascontiguousarray(q[2], np.float64)]
            self.h = lib().ipo_hip_kkt_create_q(m, n, *[_ptr(a) for a in self._keep], qmax)
        if not self.h:
            raise IpoHipError("kkt create: " + last_error())

    def factor(self, E, D):
        E = np.ascontiguousarray(E, np.float64)
        D = np.ascontiguousarray(D, np.float64)
        if lib().ipo_hip_kkt_factor(self.h, _ptr(E), _ptr(D)) != 0:
            raise IpoHipError("kkt factor: " + last_error())

    def solve(self, E, D, fy, fx):
        E = np.ascontiguousarray(E, np.float64)
        D = np.ascontiguousarray(D, np.float64)
        fy = np.array(fy, np.float64, copy=True)
        fx = np.array(fx, np.float64, copy=True)
        ok = lib().ipo_hip_kkt_solve(self.h, _ptr(E), _ptr(D), _ptr(fy), _ptr(fx))
        if ok < 0:
            raise IpoHipError("kkt solve: " + last_error())
        return fy, fx, ok

    def info(self) -> dict:
        lnz, narth, eps = C.c_long(), C.c_double(), C.c_double()
        nsup, nlev, denwin, pdf, ndep, passes = (C.c_int() for _ in range(6))
        lib().ipo_hip_kkt_info(self.h, C.byref(lnz), C.byref(narth), C.byref(nsup), C.byref(nlev), C.byref(denwin),
                               C.byref(pdf), C.byref(eps), C.byref(ndep), C.byref(passes))
        return dict(lnz=lnz.value, narth=narth.value, nsup=nsup.value, nlevels=nlev.value, denwin=denwin.value,
                    pdf=pdf.value, epsdiag=eps.value, ndep=ndep.value, passes=passes.value)

    def set_epsdiag(self, eps: float):
        lib().ipo_hip_kkt_set_epsdiag(self.h, float(eps))

    def perm(self) -> np.ndarray:
        p = np.zeros(self.m + self.n, np.int32)
        lib().ipo_hip_kkt_perm(self.h, _ptr(p))
        return p

    def pivots(self):
        """(D, live) of the last factorisation, new order."""
        d = np.zeros(self.m + self.n)
        live = np.zeros(self.m + self.n, np.int32)
        if lib().ipo_hip_kkt_pivots(self.h, _ptr(d), _ptr(live)) != 0:
            raise RuntimeError("ipo_hip_kkt_pivots failed")
        return d, live

    def close(self):
        if self.h:
            lib().ipo_hip_kkt_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """Device-resident problem (ipo_hip_ctx): setup once, run() many times."""

    def __init__(self, p: SolverForm):
        require_gpu()
        self.p = p
        self._keep = [np.ascontiguousarray(p.kA, np.int32), np.ascontiguousarray(p.iA, np.int32),
                      np.ascontiguousarray(p.A, np.float64), np.ascontiguousarray(p.b, np.float64),
                      np.ascontiguousarray(p.c, np.float64)]
        self.h = lib().ipo_hip_ctx_create(p.m, p.n, *[_ptr(a) for a in self._keep], float(p.f))
        if not self.h:
            raise IpoHipError("ctx create: " + last_error())
        self.setup_seconds = lib().ipo_hip_ctx_setup_seconds(self.h)

    def run(self, method="hsd", max_iter=200, trace=False, timing=False):
        st = Stats()

        def call(fp):
            return lib().ipo_hip_ctx_run(self.h, METHODS[method], max_iter, fp, int(timing), C.byref(st))
        if trace:
            status, text = _capture(call)
        else:
            status, text = call(None), ""
        return status, st.as_dict(), text

    def solution(self):
        x = np.zeros(self.p.n); z = np.zeros(self.p.n); y = np.zeros(self.p.m); w = np.zeros(self.p.m)
        lib().ipo_hip_ctx_download(self.h, _ptr(x), _ptr(y), _ptr(w), _ptr(z))
        return x, y, w, z

    def close(self):
        if self.h:
            lib().ipo_hip_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def set_device(device: int) -> None:
    """hipSetDevice for the library's calls from this thread (one process per GPU)."""
    if lib().ipo_hip_set_device(int(device)):
        raise IpoHipError("set_device: " + last_error())


def rccl_unique_id() -> bytes:
    """128-byte ncclUniqueId for a sharded solve; rank 0 creates it, the caller distributes it."""
    buf = C.create_string_buffer(128)
    if lib().ipo_hip_rccl_unique_id(buf):
        raise IpoHipError("rccl_unique_id: " + last_error())
    return buf.raw


def host_allreduce_callback(host_allreduce):
    """exchange.h's HostAllreduceFn around `host_allreduce(buf, op)` (a
    float64 numpy view of the staged buffer, reduced in place; op 0 sum,
    1 max, 2 min): what make_host_exchange calls between its device-to-host
    and host-to-device copies.  A raised exception returns 1, which the C
    side turns into the solve's failure.  Keep the returned object alive as
    long as the C side may call it."""
    def _allreduce(user, buf, n, op):
        try:
            host_allreduce(np.ctypeslib.as_array(buf, shape=(n,)), op)
            return 0
        except Exception:       # noqa: BLE001 -- reported through the C side's failure path
            import traceback
            traceback.print_exc()
            return 1
    return ALLREDUCE_FN(_allreduce)


class ShardContext(Context):
    """One shard of a block-angular LP on this process's GPU (ipo_hip_ctx_create_shard).

    `local` is the shard's problem from :func:`shard_block_angular` (its
    ``blocks`` carry nlink and the global sizes).  Exchange between the
    nranks shards: RCCL when `rccl_id` (rank 0's :func:`rccl_unique_id`) is
    given, else `host_allreduce(buf, op)`, called with a float64 numpy view of
    the staged data to reduce in place over all ranks (op 0 sum, 1 max,
    2 min).  nranks == 1: one process, linking rows in the dense tail.
    run() / solution() / close() as for :class:`Context`; every rank must
    call run() together."""

    def __init__(self, local, nranks: int = 1, rank: int = 0, rccl_id: bytes = None, host_allreduce=None):
        require_gpu()
        self.p = local
        self.nranks, self.rank = nranks, rank
        bl = local.blocks or {}
        self._keep = [np.ascontiguousarray(local.kA, np.int32), np.ascontiguousarray(local.iA, np.int32),
                      np.ascontiguousarray(local.A, np.float64), np.ascontiguousarray(local.b, np.float64),
                      np.ascontiguousarray(local.c, np.float64)]
        self._cb = None
        cb = None
        if rccl_id is None and host_allreduce is not None:
            self._cb = host_allreduce_callback(host_allreduce)
            cb = C.cast(self._cb, C.c_void_p)
        uid = C.create_string_buffer(bytes(rccl_id), 128) if rccl_id is not None else None
        self.h = lib().ipo_hip_ctx_create_shard(
            local.m, local.n, *[_ptr(a) for a in self._keep], float(local.f), int(bl.get("nlink", 0)),
            int(bl.get("m_global", local.m)), int(bl.get("n_global", local.n)), int(bl.get("nz_global", local.nz)),
            nranks, rank, uid, cb, None)
        if not self.h:
            raise IpoHipError("shard ctx create: " + last_error())
        self.setup_seconds = lib().ipo_hip_ctx_setup_seconds(self.h)


def symbolic(m, n, kA, iA, q=None) -> dict:
    """Host-only symbolic analysis (reference ordering); no GPU needed.
    q = (kQ, iQ[, Q]): a Q block's pattern on the y-nodes."""
    kA = np.ascontiguousarray(kA, np.int32)
    iA = np.ascontiguousarray(iA, np.int32)
    perm = np.zeros(m + n, np.int32)
    lnz, narth = C.c_long(), C.c_double()
    denwin, pdf, nsup, nlev = C.c_int(), C.c_int(), C.c_int(), C.c_int()
    kQ = iQ = None
    if q is not None:
        kQ, iQ = np.ascontiguousarray(q[0], np.int32), np.ascontiguousarray(q[1], np.int32)
    rc = lib().ipo_hip_symbolic_q(m, n, _ptr(kA), _ptr(iA), _ptr(kQ) if kQ is not None else None,
                                  _ptr(iQ) if iQ is not None else None, _ptr(perm), C.byref(lnz), C.byref(narth),
                                  C.byref(denwin), C.byref(pdf), C.byref(nsup), C.byref(nlev))
    if rc:
        raise IpoHipError("symbolic: " + last_error())
    return dict(perm=perm, lnz=lnz.value, narth=narth.value, denwin=denwin.value, pdf=pdf.value, nsup=nsup.value,
                nlevels=nlev.value)


def symbolic_forced(m, n, kA, iA, nforced) -> dict:
    """Host-only symbolic analysis with the last `nforced` rows forced into the dense tail."""
    kA = np.ascontiguousarray(kA, np.int32)
    iA = np.ascontiguousarray(iA, np.int32)
    perm = np.zeros(m + n, np.int32)
    cc = np.zeros(m + n, np.int32)
    lnz, tc, nsup, nlev = C.c_long(), C.c_int(), C.c_int(), C.c_int()
    rc = lib().ipo_hip_symbolic_forced(m, n, _ptr(kA), _ptr(iA), nforced, _ptr(perm), _ptr(cc), C.byref(lnz),
                                       C.byref(tc), C.byref(nsup), C.byref(nlev))
    if rc:
        raise IpoHipError("symbolic_forced: " + last_error())
    return dict(perm=perm, colcount=cc, lnz=lnz.value, tail_c0=tc.value, nsup=nsup.value, nlevels=nlev.value)


# ----------------------------------------------------------------- synthetic LPs
SYNTH_SEED = 20251121


@dataclass
class SynthProblem(SolverForm):
    """A synthetic LP plus the interior point it was generated from."""
    xs: np.ndarray = None
    ys: np.ndarray = None
    ws: np.ndarray = None
    zs: np.ndarray = None
    blocks: dict = None


def _synth_arrays(m, n, nz):
    return (np.zeros(n + 1, np.int32), np.zeros(nz, np.int32), np.zeros(nz), np.zeros(m), np.zeros(n),
            np.zeros(n), np.zeros(m), np.zeros(m), np.zeros(n))


def synth_random(m, n, per_col=4, band=0, seed=SYNTH_SEED) -> SynthProblem:
    """BASELINE configs[3]: random sparse LP (band=0 uniform rows, band>0 banded)."""
    nz = C.c_int(0)
    L = lib()
    if L.ipo_hip_synth_random(m, n, per_col, band, seed, C.byref(nz), *([None] * 9)):
        raise IpoHipError("synth_random: " + last_error())
    arrs = _synth_arrays(m, n, nz.value)
    kA, iA, A, b, c, xs, ys, ws, zs = arrs
    if L.ipo_hip_synth_random(m, n, per_col, band, seed, C.byref(nz), *[_ptr(a) for a in arrs]):
        raise IpoHipError("synth_random: " + last_error())
    return SynthProblem(m, n, kA, iA, A, b, c, 0.0, xs, ys, ws, zs)


VECTOR_KERNELS = ("k_hsd_residuals", "k_hsd_directions", "k_step")


def dot_ordered(a, b) -> float:
    """The solver's ordered dot of two float64 vectors on the GPU (test entry)."""
    require_gpu()
    a = np.ascontiguousarray(a, np.float64)
    b = np.ascontiguousarray(b, np.float64)
    out = np.zeros(1, np.float64)
    if lib().ipo_hip_dot_ordered(_ptr(a), _ptr(b), int(a.size), _ptr(out)):
        raise IpoHipError("dot_ordered: " + last_error())
    return float(out[0])


def vector_bench(p, reps=20) -> dict:
    """Time the HBM-bound HSD vector kernels alone on LP p (device-resident
    inputs): {kernel: (ms per launch, algorithmic bytes per launch)}."""
    require_gpu()
    ms, by = np.zeros(3), np.zeros(3)
    kA = np.ascontiguousarray(p.kA, np.int32)
    iA = np.ascontiguousarray(p.iA, np.int32)
    A = np.ascontiguousarray(p.A, np.float64)
    if lib().ipo_hip_vector_bench(p.m, p.n, _ptr(kA), _ptr(iA), _ptr(A), reps, _ptr(ms), _ptr(by)):
        raise IpoHipError("vector_bench: " + last_error())
    return {k: (float(ms[i]), float(by[i])) for i, k in enumerate(VECTOR_KERNELS)}


def synth_block_angular(nblocks=8, mb=25000, nb=100000, per_col=4, band=256, nlink=512, link_nz=2000,
                        seed=SYNTH_SEED) -> SynthProblem:
    """BASELINE configs[4]: block-angular LP, linking rows last."""
    m, n, nz = C.c_int(0), C.c_int(0), C.c_int(0)
    L = lib()
    args = (nblocks, mb, nb, per_col, band, nlink, link_nz, seed, C.byref(m), C.byref(n), C.byref(nz))
    if L.ipo_hip_synth_block_angular(*args, *([None] * 9)):
        raise IpoHipError("synth_block_angular: " + last_error())
    arrs = _synth_arrays(m.value, n.value, nz.value)
    kA, iA, A, b, c, xs, ys, ws, zs = arrs
    if L.ipo_hip_synth_block_angular(*args, *[_ptr(a) for a in arrs]):
        raise IpoHipError("synth_block_angular: " + last_error())
    return SynthProblem(m.value, n.value, kA, iA, A, b, c, 0.0, xs, ys, ws, zs,
                        dict(nblocks=nblocks, mb=mb, nb=nb, nlink=nlink))


def shard_block_angular(p: SynthProblem, nshards: int, k: int) -> SynthProblem:
    """Local LP of shard k of a block-angular problem.

    Shard k owns the diagonal blocks [k B/nshards, (k+1) B/nshards) -- their
    rows and columns -- plus a replica of every linking row, numbered after
    its own rows.  Its A is the column slice restricted to those rows; b of
    the linking rows and every linking-row quantity are replicated on all
    shards.  Returns the local problem (blocks: row/column offsets in the
    global problem)."""
    B = p.blocks["nblocks"]
    mb, nb, nl = p.blocks["mb"], p.blocks["nb"], p.blocks["nlink"]
    if B % nshards:
        raise IpoHipError(f"{B} blocks do not split evenly over {nshards} shards")
    per = B // nshards
    r0, r1 = k * per * mb, (k + 1) * per * mb
    c0, c1 = k * per * nb, (k + 1) * per * nb
    mloc = r1 - r0 + nl
    kA = (p.kA[c0:c1 + 1] - p.kA[c0]).astype(np.int32)
    rows = p.iA[p.kA[c0]:p.kA[c1]]
    iA = np.where(rows >= B * mb, rows - B * mb + (r1 - r0), rows - r0).astype(np.int32)
    A = p.A[p.kA[c0]:p.kA[c1]].copy()
    b = np.concatenate([p.b[r0:r1], p.b[B * mb:]])
    c = p.c[c0:c1].copy()
    ys = np.concatenate([p.ys[r0:r1], p.ys[B * mb:]]) if p.ys is not None else None
    ws = np.concatenate([p.ws[r0:r1], p.ws[B * mb:]]) if p.ws is not None else None
    return SynthProblem(mloc, c1 - c0, kA, iA, A, b, c, 0.0,
                        p.xs[c0:c1].copy() if p.xs is not None else None, ys, ws,
                        p.zs[c0:c1].copy() if p.zs is not None else None,
                        dict(nblocks=per, mb=mb, nb=nb, nlink=nl, row0=r0, col0=c0, shard=k, nshards=nshards,
                             m_global=p.m, n_global=p.n, nz_global=p.nz))


def assemble_block_angular(parts):
    """Global (x, y, w, z) of a sharded solve from every shard's (blocks, (x, y, w, z)).

    Columns and block rows concatenate in shard order; the linking rows are
    replicated on every shard and taken from shard 0."""
    parts = sorted(parts, key=lambda t: t[0]["shard"])
    nl = parts[0][0]["nlink"]
    x = np.concatenate([s[0] for _, s in parts])
    z = np.concatenate([s[3] for _, s in parts])
    y = np.concatenate([s[1][:len(s[1]) - nl] for _, s in parts] + [parts[0][1][1][len(parts[0][1][1]) - nl:]])
    w = np.concatenate([s[2][:len(s[2]) - nl] for _, s in parts] + [parts[0][1][2][len(parts[0][1][2]) - nl:]])
    return x, y, w, z
