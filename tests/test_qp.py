"""The Q block of the reference's KKT system, host side.

ldlt.c factors K = [ -(Q + dn)  A' ; A  dm ] with lp->Q on its first node
class (ldlt.c:253-256) and carries max Q x in its refinement residual
(ldlt.c:391-394); the MPS reader keeps QUADS (iolp.c:583-645) and
symmetrises it (iolp.c:733-793).  ipo's own solvers never set Q
(ldlt.c:142-144 allocates it empty; solve.c:24-26 has no Q), and the
reference holds no QP fixture, so parity here is against the oracle's
restatement of the same lines ("parity unpinned" by reference output):

  * the reader: the product's QUADS (lp_io.cpp) and the oracle's
    (orc_mps.c) identical on QP files written here, entries above the
    diagonal ignored (iolp.c:618 warn 35), columns out of order rejected (36);
  * the ordering with Q: the reference's tiered minimum degree with the Q
    neighbours appended to each y-node's adjacency (ldlt.c:729-745) and
    the primal priority refused for a non-separable Q (ldlt.c:675-682, 710):
    the product's permutation, lnz, narth and priority identical to the
    oracle's.
The numeric factor and refined solve with Q run on the GPU
(tests/test_gpu_qp.py)."""
import os

import numpy as np
import pytest

import ipo_amd
import oracle_lib
from conftest import mps_path


def random_q(m, seed, band=6, density=0.5, diag=True):
    """A symmetric, diagonally dominant (positive definite) Q on m nodes:
    off-diagonal entries within `band` of the diagonal, full symmetric CSC
    with rows sorted (the layout iolp.c:733-793 leaves)."""
    rng = np.random.default_rng(seed)
    ent = {}
    for j in range(m):
        for i in range(j + 1, min(m, j + band + 1)):
            if rng.random() < density:
                v = rng.uniform(-1, 1)
                ent[(i, j)] = v
                ent[(j, i)] = v
    rowsum = np.zeros(m)
    for (i, j), v in ent.items():
        rowsum[i] += abs(v)
    if diag:
        for j in range(m):
            ent[(j, j)] = rowsum[j] + rng.uniform(0.5, 1.5)
    kQ = np.zeros(m + 1, np.int32)
    cols = [[] for _ in range(m)]
    for (i, j), v in ent.items():
        cols[j].append((i, v))
    iQ, Q = [], []
    for j in range(m):
        cols[j].sort()
        iQ += [i for i, _ in cols[j]]
        Q += [v for _, v in cols[j]]
        kQ[j + 1] = len(iQ)
    return kQ, np.array(iQ, np.int32), np.array(Q, np.float64)


# ---------------------------------------------------------------- QUADS reader
def _card(kind, n0, n1="", v1=None, n2="", v2=None):
    """One fixed-column MPS card (fields at columns 2, 5, 15, 25, 40, 50)."""
    s = f" {kind:<2} {n0:<8}  {n1:<8}  {'' if v1 is None else repr(v1):>12}"
    if n2:
        s += f"   {n2:<8}  {repr(v2):>12}"
    return s.rstrip() + "\n"


QP_MPS = ("NAME          QPTEST\nROWS\n N  COST\n L  LIM1\n G  LIM2\n E  MYEQN\nCOLUMNS\n"
          + _card("", "X1", "COST", 1.0, "LIM1", 1.0) + _card("", "X1", "LIM2", 1.0)
          + _card("", "X2", "COST", 2.0, "LIM1", 1.0) + _card("", "X2", "MYEQN", -1.0)
          + _card("", "X3", "COST", -1.0, "MYEQN", 1.0) + _card("", "X4", "COST", 0.5, "LIM2", 1.0)
          + "RHS\n" + _card("", "RHS", "LIM1", 4.0, "LIM2", 1.0) + _card("", "RHS", "MYEQN", 7.0)
          + "BOUNDS\n" + _card("UP", "BND", "X1", 4.0)
          + "QUADS\n" + _card("", "X1", "X1", 2.0, "X2", 0.5) + _card("", "X1", "X4", -0.25)
          + _card("", "X2", "X2", 3.0, "X1", 9.0) + _card("", "X3", "X3", 1.5) + _card("", "X4", "X4", 1.0)
          + "ENDATA\n")


def _write(tmp_path, text, name="qp.mps"):
    p = os.path.join(tmp_path, name)
    with open(p, "w") as fh:
        fh.write(text)
    return p


def _orc_quads(path):
    import ctypes as C
    L = oracle_lib.lib()
    L.orc_mps_quads.argtypes = [C.c_char_p] + [C.c_void_p] * 5
    L.orc_mps_quads.restype = C.c_int
    n, qnz = C.c_int(), C.c_int()
    rc = L.orc_mps_quads(path.encode(), C.addressof(n), C.addressof(qnz), None, None, None)
    if rc:
        return rc
    if qnz.value < 0:
        return None
    kQ = np.zeros(n.value + 1, np.int32)
    iQ = np.zeros(max(1, qnz.value), np.int32)
    Q = np.zeros(max(1, qnz.value), np.float64)
    L.orc_mps_quads(path.encode(), None, None, kQ.ctypes.data, iQ.ctypes.data, Q.ctypes.data)
    return kQ, iQ[:qnz.value], Q[:qnz.value]


def test_quads_reader_matches_oracle(tmp_path):
    path = _write(str(tmp_path), QP_MPS)
    mine = ipo_amd.mps_quads(path)
    ref = _orc_quads(path)
    for a, b in zip(mine, ref):
        assert np.array_equal(a, b)
    kQ, iQ, Q = mine
    dense = np.zeros((4, 4))
    for j in range(4):
        dense[iQ[kQ[j]:kQ[j + 1]], j] = Q[kQ[j]:kQ[j + 1]]
    # X1 X2 0.5 and X1 X4 -0.25 below the diagonal, mirrored; the diagonal;
    # "X2 X1 9.0" lies above the diagonal (row X1 < column X2): ignored
    expect = np.array([[2.0, 0.5, 0.0, -0.25], [0.5, 3.0, 0.0, 0.0], [0.0, 0.0, 1.5, 0.0], [-0.25, 0.0, 0.0, 1.0]])
    assert np.array_equal(dense, expect)
    for j in range(4):
        assert np.all(np.diff(iQ[kQ[j]:kQ[j + 1]]) > 0)


def test_quads_absent_and_out_of_order(tmp_path):
    assert ipo_amd.mps_quads(mps_path("afiro")) is None
    assert _orc_quads(mps_path("afiro")) is None
    a, b = _card("", "X3", "X3", 1.5), _card("", "X4", "X4", 1.0)
    bad = QP_MPS.replace(a + b, b + a)
    assert bad != QP_MPS
    path = _write(str(tmp_path), bad, "bad.mps")
    with pytest.raises(ipo_amd.IpoHipError, match="36"):
        ipo_amd.mps_quads(path)
    assert _orc_quads(path) == 36


def test_quads_do_not_change_the_lp(tmp_path):
    """solve.c has no Q: the problem handed to solver() is the LP's."""
    path = _write(str(tmp_path), QP_MPS)
    lp = _write(str(tmp_path), QP_MPS.split("QUADS")[0] + "ENDATA\n", "lp.mps")
    a, b = ipo_amd.load_mps(path), ipo_amd.load_mps(lp)
    assert (a.m, a.n) == (b.m, b.n)
    for x, y in ((a.kA, b.kA), (a.iA, b.iA), (a.A, b.A), (a.b, b.b), (a.c, b.c)):
        assert np.array_equal(x, y)


# ---------------------------------------------------------------- ordering with Q
QNAMES = ["afiro", "blend", "sc50a", "kb2", "share2b", "israel", "bandm", "25fv47"]


@pytest.mark.parametrize("name", QNAMES)
@pytest.mark.parametrize("diag_only", [False, True])
def test_ordering_with_q_matches_oracle(name, diag_only):
    p = ipo_amd.load_mps(mps_path(name))
    q = random_q(p.m, 11, band=0 if diag_only else 6)
    mine = ipo_amd.symbolic(p.m, p.n, p.kA, p.iA, q=q)
    ok = oracle_lib.OracleKkt(p, q=q, qmax=1)
    ref = ok.info()
    assert np.array_equal(mine["perm"], ok.perm())
    assert mine["lnz"] == ref["lnz"] and mine["narth"] == ref["narth"] and mine["pdf"] == ref["pdf"]
    if not diag_only:
        assert ref["pdf"] == 2          # not separable: dual priority (ldlt.c:710)
    if diag_only:                       # a diagonal Q adds no edge: the LP's own ordering
        assert np.array_equal(mine["perm"], ipo_amd.symbolic(p.m, p.n, p.kA, p.iA)["perm"])


def test_oracle_factor_with_q_solves_the_qp_system():
    """The oracle's K with Q satisfies the QP KKT system to the refinement
    target (a self-check of the restatement before the GPU is held to it)."""
    import scipy.sparse as sp
    p = ipo_amd.load_mps(mps_path("afiro"))
    q = random_q(p.m, 3)
    rng = np.random.default_rng(5)
    E, D = rng.uniform(0.1, 10, p.m), rng.uniform(0.1, 10, p.n)
    fy, fx = rng.uniform(-1, 1, p.m), rng.uniform(-1, 1, p.n)
    for qmax in (1, -1):
        o = oracle_lib.OracleKkt(p, q=q, qmax=qmax)
        o.factor(E, D)
        dy, dx, ok = o.solve(E, D, fy, fx)
        A = sp.csc_matrix((p.A, p.iA, p.kA), shape=(p.m, p.n))
        Qm = sp.csc_matrix((q[2], q[1], q[0]), shape=(p.m, p.m))
        ry = fy - (A @ dx - E * dy - qmax * (Qm @ dy))
        rx = fx - (A.T @ dy + D * dx)
        assert max(np.abs(ry).max(), np.abs(rx).max()) <= 1e-9 * (1 + max(np.abs(fy).max(), np.abs(fx).max()))


def test_set_q_validates_input():
    """ipo_hip_ldlt_set_q (host only: no device until ldltfac) refuses a Q
    the header's contract excludes -- rows out of range, unsorted or
    duplicated rows in a column, an asymmetric pattern or value -- with -1
    and a message, and accepts a valid one."""
    import ctypes as C
    L = ipo_amd.lib()
    L.ipo_hip_ldlt_set_q.argtypes = [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int]
    L.ipo_hip_ldlt_set_q.restype = C.c_int
    L.inv_clo.restype = None

    def setq(kQ, iQ, Q, n=None):
        kQ, iQ, Q = (np.ascontiguousarray(kQ, np.int32), np.ascontiguousarray(iQ, np.int32),
                     np.ascontiguousarray(Q, np.float64))
        n = len(kQ) - 1 if n is None else n
        rc = L.ipo_hip_ldlt_set_q(n, kQ.ctypes.data, iQ.ctypes.data, Q.ctypes.data, 1)
        L.inv_clo()
        return rc, ipo_amd.last_error()

    kQ, iQ, Q = random_q(12, 3)
    assert setq(kQ, iQ, Q)[0] == 0
    bad_row = iQ.copy(); bad_row[2] = 12
    rc, msg = setq(kQ, bad_row, Q)
    assert rc == -1 and "out of range" in msg
    j = next(j for j in range(12) if kQ[j + 1] - kQ[j] >= 2)
    unsorted = iQ.copy(); unsorted[kQ[j]], unsorted[kQ[j] + 1] = unsorted[kQ[j] + 1], unsorted[kQ[j]]
    rc, msg = setq(kQ, unsorted, Q)
    assert rc == -1 and "ascending" in msg
    asym = Q.copy()
    k = next(k for k in range(kQ[j], kQ[j + 1]) if iQ[k] != j)
    asym[k] += 1.0
    rc, msg = setq(kQ, iQ, asym)
    assert rc == -1 and "symmetric" in msg
    # diagonal only, one column without its twin: (1, 0) present, (0, 1) absent
    rc, msg = setq([0, 2, 3], [0, 1, 1], [1.0, 0.5, 1.0])
    assert rc == -1 and "symmetric" in msg
