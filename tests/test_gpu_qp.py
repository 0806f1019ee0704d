"""The Q block of the reference's KKT system on the GPU.

K = [ -(max(E, eps) + qmax Q)  A ; A'  max(D, eps) ]: -qmax Q assembled into
the y-node block (ldlt.c:253-256, the block of ldlt.c's dn), qmax Q dy in the
refinement residual (ldlt.c:391-394).  Against the oracle's restatement of
the same lines (orc_kkt_create_q; the reference holds no QP fixture, so the
parity is pinned by the oracle only) on identical inputs -- same ordering,
fill pattern and operations in another summation order:
  * the permutation identical (the reference's ordering with Q);
  * the pivots D within 1e-9 relative (the LP tolerance of test_gpu_kkt.py);
  * the refined solution within 1e-8 x (1 + |x|) and the QP KKT residual
    within 1e-9 of the right-hand side scale;
  * through the LU plug-in (ldltfac / forwardbackward with the reference's
    swapped roles, Q attached by ipo_hip_ldlt_set_q) the same;
  * the nested-dissection order with a Q (its graph no longer bipartite)
    solves the same system to the same tolerance."""
import numpy as np
import pytest
import scipy.sparse as sp

import ipo_amd
import oracle_lib
from conftest import mps_path
from test_qp import random_q

pytestmark = pytest.mark.gpu

NAMES = ["afiro", "blend", "sc50a", "share2b", "israel", "bandm", "25fv47", "d6cube"]


def qp_residual(p, q, qmax, E, D, fy, fx, dy, dx):
    A = sp.csc_matrix((p.A, p.iA, p.kA), shape=(p.m, p.n))
    Qm = sp.csc_matrix((q[2], q[1], q[0]), shape=(p.m, p.m))
    ry = fy - (A @ dx - E * dy - qmax * (Qm @ dy))
    rx = fx - (A.T @ dy + D * dx)
    return max(np.abs(ry).max(initial=0), np.abs(rx).max(initial=0))


def _inputs(p, seed):
    rng = np.random.default_rng(seed)
    return (rng.uniform(0.1, 10.0, p.m), rng.uniform(0.1, 10.0, p.n), rng.uniform(-1, 1, p.m),
            rng.uniform(-1, 1, p.n))


@pytest.mark.parametrize("name", NAMES)
@pytest.mark.parametrize("qmax", [1, -1])
def test_kkt_with_q_matches_oracle(name, qmax):
    p = ipo_amd.load_mps(mps_path(name))
    q = random_q(p.m, 17)
    E, D, fy, fx = _inputs(p, 20251121)
    if qmax < 0:
        E = E + 2 * q[2].max()          # keep -E + Q negative definite (quasi-definite K)
    gpu = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A, q=q, qmax=qmax)
    orc = oracle_lib.OracleKkt(p, q=q, qmax=qmax)
    try:
        assert np.array_equal(gpu.perm(), orc.perm())
        gpu.factor(E, D)
        orc.factor(E, D)
        gd, glive = gpu.pivots()
        od = orc.diag()
        assert np.array_equal(glive, orc.live()) and gpu.info()["ndep"] == orc.info()["ndep"] == 0
        assert (np.abs(gd - od) <= 1e-9 * np.abs(od)).all()
        gy, gx, ok = gpu.solve(E, D, fy, fx)
        oy, ox, _ = orc.solve(E, D, fy, fx)
        assert ok == 1
        scale = 1.0 + max(np.abs(oy).max(), np.abs(ox).max())
        assert np.abs(gy - oy).max() <= 1e-8 * scale and np.abs(gx - ox).max() <= 1e-8 * scale
        bc = max(np.abs(fy).max(), np.abs(fx).max()) + 1
        assert qp_residual(p, q, qmax, E, D, fy, fx, gy, gx) <= 1e-9 * bc
    finally:
        gpu.close()


def test_ldltfac_plugin_with_q():
    """ldltfac / forwardbackward (ldlt.h) with the reference's swapped roles
    (hsd.c:218: ldltfac(n, m, kAt, iAt, At, E, D, kA, iA, A, v)), the Q block
    on ldltfac's n-block -- the block of dn = E -- set before the first call."""
    p = ipo_amd.load_mps(mps_path("afiro"))
    q = random_q(p.m, 4)
    kAt, iAt, At = p.transpose()
    E, D, fy, fx = _inputs(p, 3)
    L = ipo_amd.lib()
    kA, iA, A = p.kA.astype(np.int32), p.iA.astype(np.int32), p.A.copy()
    kQ, iQ, Qv = (np.ascontiguousarray(a) for a in q)
    assert L.ipo_hip_ldlt_set_q(p.m, kQ.ctypes.data, iQ.ctypes.data, Qv.ctypes.data, 1) == 0
    try:
        L.ldltfac(p.n, p.m, kAt.ctypes.data, iAt.ctypes.data, At.ctypes.data, E.ctypes.data, D.ctypes.data,
                  kA.ctypes.data, iA.ctypes.data, A.ctypes.data, 1)
        assert L.ipo_hip_ldlt_set_q(p.m, kQ.ctypes.data, iQ.ctypes.data, Qv.ctypes.data, 1) == -1   # after ldltfac
        y = fy.copy()
        x = fx.copy()
        L.forwardbackward(E.ctypes.data, D.ctypes.data, y.ctypes.data, x.ctypes.data)
    finally:
        L.inv_clo()
    orc = oracle_lib.OracleKkt(p, q=q, qmax=1)
    orc.factor(E, D)
    oy, ox, _ = orc.solve(E, D, fy, fx)
    assert np.allclose(y, oy, rtol=1e-9, atol=1e-10) and np.allclose(x, ox, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("leaf", [16, 1024])
def test_nested_dissection_with_q(monkeypatch, leaf):
    monkeypatch.setenv("IPO_HIP_ORDER", "nd")
    monkeypatch.setenv("IPO_HIP_ND_LEAF", str(leaf))
    p = ipo_amd.synth_random(2000, 10000, 4, 64)
    q = random_q(p.m, 9, band=8)
    E, D, fy, fx = _inputs(p, 8)
    gpu = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A, q=q, qmax=1)
    try:
        gpu.factor(E, D)
        gy, gx, ok = gpu.solve(E, D, fy, fx)
    finally:
        gpu.close()
    orc = oracle_lib.OracleKkt(p, q=q, qmax=1)
    orc.factor(E, D)
    oy, ox, _ = orc.solve(E, D, fy, fx)
    assert ok == 1
    scale = 1.0 + max(np.abs(oy).max(), np.abs(ox).max())
    assert np.abs(gy - oy).max() <= 1e-8 * scale and np.abs(gx - ox).max() <= 1e-8 * scale
    bc = max(np.abs(fy).max(), np.abs(fx).max()) + 1
    assert qp_residual(p, q, 1, E, D, fy, fx, gy, gx) <= 1e-9 * bc
