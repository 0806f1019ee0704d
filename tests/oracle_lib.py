"""Test-side access to the CPU ORACLE (oracle/, test infrastructure only).

Builds oracle/ with its Makefile on first use and exposes the CLI (full
`ipo` stdout) and the KKT LDL' pieces through ctypes.  Never imported by
the product (linear-programming-vanderbei_amd/)."""
import ctypes as C
import os
import subprocess
import threading

import numpy as np

from conftest import REPO

ORACLE_DIR = os.path.join(REPO, "oracle")
BUILD = os.path.join(ORACLE_DIR, "build")
_lock = threading.Lock()
_lib = None


def build():
    with _lock:
        subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)


def cli_path():
    exe = os.path.join(BUILD, "ipo_oracle")
    if not os.path.exists(exe):
        build()
    return exe


def run_cli(mps: str, method: str = "hsd", timeout: float = 3600, free: str = "abort", solfile: str = None) -> str:
    """The oracle's `ipo` stdout.  free="split": the free-variable extension
    (orc_split_free); solfile: its writesol report there."""
    env = dict(os.environ)
    if free == "split":
        env["ORC_FREE"] = "1"
    if solfile:
        env["ORC_SOLFILE"] = solfile
    out = subprocess.run([cli_path(), mps, method], capture_output=True, text=True, timeout=timeout, env=env)
    return out.stdout


def write_sol(mps: str, x, y, z, solfile: str) -> int:
    """orc_writesol_mps: the oracle's writesol restatement from solver()-form vectors."""
    L = lib()
    L.orc_writesol_mps.argtypes = [C.c_char_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_char_p]
    L.orc_writesol_mps.restype = C.c_int
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    z = np.ascontiguousarray(z, np.float64)
    return L.orc_writesol_mps(mps.encode(), x.ctypes.data, y.ctypes.data, z.ctypes.data, solfile.encode())


def lib():
    global _lib
    if _lib is None:
        so = os.path.join(BUILD, "liborc.so")
        if not os.path.exists(so):
            build()
        L = C.CDLL(so)
        P, I, D = C.c_void_p, C.c_int, C.c_double
        L.orc_kkt_create.restype = P
        L.orc_kkt_create.argtypes = [I, I, P, P, P, P, P, P]
        L.orc_kkt_create_q.restype = P
        L.orc_kkt_create_q.argtypes = [I, I, P, P, P, P, P, P, P, P, P, I]
        L.orc_kkt_destroy.argtypes = [P]
        L.orc_kkt_factor.argtypes = [P, P, P]
        L.orc_kkt_solve.argtypes = [P, P, P, P, P]
        L.orc_kkt_solve.restype = I
        L.orc_kkt_lnz.restype = C.c_long
        L.orc_kkt_lnz.argtypes = [P]
        L.orc_kkt_narth.restype = D
        L.orc_kkt_narth.argtypes = [P]
        for f in ("orc_kkt_denwin", "orc_kkt_pdf", "orc_kkt_dim", "orc_kkt_ndep", "orc_kkt_last_passes"):
            getattr(L, f).argtypes = [P]
            getattr(L, f).restype = I
        L.orc_kkt_epsdiag.restype = D
        L.orc_kkt_epsdiag.argtypes = [P]
        L.orc_kkt_perm.argtypes = [P, P]
        L.orc_kkt_diag.argtypes = [P, P]
        L.orc_kkt_live.argtypes = [P, P]
        L.orc_set_perturb.argtypes = [I]
        L.orc_set_perturb.restype = None
        L.orc_kkt_set_epsdiag.argtypes = [P, D]
        _lib = L
    return _lib


class OracleKkt:
    """orc_kkt: the reference's tiered-MD ordering + left-looking LDL'."""

    def __init__(self, form, q=None, qmax=1):
        """q = (kQ, iQ, Q): the Q block on the y-nodes (m x m, full symmetric
        CSC), K_yy = -max(E, eps) - qmax Q (orc_kkt_create_q)."""
        L = lib()
        self.m, self.n = form.m, form.n
        kAt, iAt, At = form.transpose()
        self._keep = [np.ascontiguousarray(form.kA, np.int32), np.ascontiguousarray(form.iA, np.int32),
                      np.ascontiguousarray(form.A, np.float64), kAt, iAt, At]
        if q is None:
            self.h = L.orc_kkt_create(self.m, self.n, *[a.ctypes.data for a in self._keep])
        else:
            self._keep += [np.ascontiguousarray(q[0], np.int32), np.ascontiguousarray(q[1], np.int32),
                           np.ascontiguousarray(q[2], np.float64)]
            self.h = L.orc_kkt_create_q(self.m, self.n, *[a.ctypes.data for a in self._keep], qmax)

    def factor(self, E, D):
        E = np.ascontiguousarray(E, np.float64)
        D = np.ascontiguousarray(D, np.float64)
        lib().orc_kkt_factor(self.h, E.ctypes.data, D.ctypes.data)

    def solve(self, E, D, fy, fx):
        E = np.ascontiguousarray(E, np.float64)
        D = np.ascontiguousarray(D, np.float64)
        fy = np.array(fy, np.float64, copy=True)
        fx = np.array(fx, np.float64, copy=True)
        ok = lib().orc_kkt_solve(self.h, E.ctypes.data, D.ctypes.data, fy.ctypes.data, fx.ctypes.data)
        return fy, fx, ok

    def info(self):
        L = lib()
        return dict(lnz=L.orc_kkt_lnz(self.h), narth=L.orc_kkt_narth(self.h), denwin=L.orc_kkt_denwin(self.h),
                    pdf=L.orc_kkt_pdf(self.h), ndep=L.orc_kkt_ndep(self.h), epsdiag=L.orc_kkt_epsdiag(self.h),
                    passes=L.orc_kkt_last_passes(self.h))

    def set_epsdiag(self, eps):
        lib().orc_kkt_set_epsdiag(self.h, float(eps))

    def perm(self):
        p = np.zeros(self.m + self.n, np.int32)
        lib().orc_kkt_perm(self.h, p.ctypes.data)
        return p

    def live(self):
        v = np.zeros(self.m + self.n, np.int32)
        lib().orc_kkt_live(self.h, v.ctypes.data)
        return v

    def diag(self):
        d = np.zeros(self.m + self.n, np.float64)
        lib().orc_kkt_diag(self.h, d.ctypes.data)
        return d

    def __del__(self):
        try:
            lib().orc_kkt_destroy(self.h)
        except Exception:
            pass


class _OrcRun(C.Structure):
    _fields_ = [("trace", C.c_void_p), ("max_iter", C.c_int), ("iters", C.c_int), ("t_setup", C.c_double),
                ("t_total", C.c_double), ("final_mu", C.c_double), ("final_pobj", C.c_double),
                ("final_dobj", C.c_double), ("final_pinf", C.c_double), ("final_dinf", C.c_double)]


def solve_arrays(form, method="hsd", max_iter=200):
    """orc_hsd / orc_intpt / orc_hsdls on a solver()-form problem (silent).
    Returns dict(status, iters, x, y, w, z, final_*)."""
    L = lib()
    fn = {"hsd": L.orc_hsd, "intpt": L.orc_intpt, "hsdls": L.orc_hsdls}[method]
    fn.restype = C.c_int
    fn.argtypes = [C.c_int] * 3 + [C.c_void_p] * 5 + [C.c_double] + [C.c_void_p] * 4 + [C.POINTER(_OrcRun)]
    m, n = form.m, form.n
    kA = np.ascontiguousarray(form.kA, np.int32)
    iA = np.ascontiguousarray(form.iA, np.int32)
    A = np.ascontiguousarray(form.A, np.float64)
    b = np.ascontiguousarray(form.b, np.float64)
    c = np.ascontiguousarray(form.c, np.float64)
    x, z = np.zeros(n + m), np.zeros(n)
    y, w = np.zeros(n + m), np.zeros(m)
    run = _OrcRun(None, max_iter, 0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0)
    st = fn(m, n, int(kA[-1]), iA.ctypes.data, kA.ctypes.data, A.ctypes.data, b.ctypes.data, c.ctypes.data,
            float(form.f), x.ctypes.data, y.ctypes.data, w.ctypes.data, z.ctypes.data, C.byref(run))
    return dict(status=st, iters=run.iters, x=x[:n], y=y[:m], w=w, z=z, final_mu=run.final_mu,
                final_pobj=run.final_pobj, final_dobj=run.final_dobj, final_pinf=run.final_pinf,
                final_dinf=run.final_dinf)
