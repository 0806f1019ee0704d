"""HIP KKT factor + refined solve (kkt_device.hip) vs the oracle's
left-looking LDL' on identical K(E, D) -- same ordering, same fill pattern,
different summation order.

Tolerance: after iterative refinement both solutions satisfy the KKT system
to the reference's refinement target, so their difference is bounded by the
conditioning of K.  We require  ||x_gpu - x_orc||_inf <= 1e-8 * (1 + ||x_orc||_inf)
on well-scaled (E, D) and an equally small KKT residual."""
import os

import numpy as np
import pytest

import ipo_amd
import oracle_lib
from conftest import GOLDEN, mps_path

pytestmark = pytest.mark.gpu

NAMES = ["afiro", "adlittle", "blend", "sc50a", "kb2", "share2b", "israel", "bandm", "ship04s", "25fv47", "degen2",
         "d6cube", "grow22", "pds-02", "dfl001"]


def kkt_residual(p, E, D, fy, fx, dy, dx):
    import scipy.sparse as sp
    A = sp.csc_matrix((p.A, p.iA, p.kA), shape=(p.m, p.n))
    ry = fy - (A @ dx - E * dy)
    rx = fx - (A.T @ dy + D * dx)
    return max(np.abs(ry).max(initial=0), np.abs(rx).max(initial=0))


@pytest.mark.parametrize("name", NAMES)
def test_factor_solve_matches_oracle(name):
    p = ipo_amd.load_mps(mps_path(name))
    rng = np.random.default_rng(20251121)
    E = rng.uniform(0.1, 10.0, p.m)
    D = rng.uniform(0.1, 10.0, p.n)
    fy = rng.uniform(-1, 1, p.m)
    fx = rng.uniform(-1, 1, p.n)
    gpu = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
    orc = oracle_lib.OracleKkt(p)
    gpu.factor(E, D)
    orc.factor(E, D)
    assert np.array_equal(gpu.perm(), orc.perm())
    gy, gx, ok = gpu.solve(E, D, fy, fx)
    oy, ox, _ = orc.solve(E, D, fy, fx)
    assert ok == 1
    scale = 1.0 + max(np.abs(oy).max(), np.abs(ox).max())
    assert np.abs(gy - oy).max() <= 1e-8 * scale
    assert np.abs(gx - ox).max() <= 1e-8 * scale
    bc = max(np.abs(fy).max(), np.abs(fx).max()) + 1
    assert kkt_residual(p, E, D, fy, fx, gy, gx) <= 1e-9 * bc
    gi, oi = gpu.info(), orc.info()
    assert gi["lnz"] == oi["lnz"] and gi["ndep"] == oi["ndep"] == 0
    # pivot by pivot (D of the factor, new order): same operations in another
    # summation order, so relative 1e-9 on these well-scaled systems (measured
    # <= 7e-12, d6cube); every pivot live on both sides
    gd, glive = gpu.pivots()
    od = orc.diag()
    assert np.array_equal(glive, orc.live())
    assert (np.abs(gd - od) <= 1e-9 * np.abs(od)).all(), np.argmax(np.abs(gd - od) / np.abs(od))


def oracle_variants(p, E, D, eps, fy=None, fx=None):
    """The oracle under its three summation orders (orc_set_perturb:
    lltnum's order, reversed, by source column): (ndep, live, pivots,
    refined solution of (fy, fx) or None) per order."""
    L = oracle_lib.lib()
    out = []
    try:
        for order in (0, 1, 2):
            L.orc_set_perturb(order)
            o = oracle_lib.OracleKkt(p)
            o.set_epsdiag(eps)
            o.factor(E, D)
            sol = o.solve(E, D, fy, fx)[:2] if fy is not None else None
            out.append((o.info()["ndep"], o.live().copy(), o.diag().copy(), sol))
    finally:
        L.orc_set_perturb(0)
    return out


def _rel(a, b):
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-300)


STATES = sorted(f[:-4] for f in os.listdir(os.path.join(GOLDEN, "..", "kkt_states")) if f.endswith(".npz"))


@pytest.mark.parametrize("state", STATES)
def test_ipm_states_match_oracle(state):
    """Scalings captured from the oracle's own HSD runs (tools/capture_kkt_states.py),
    including late iterations with dependent rows and a grown eps_diag.
    Tolerance:
      * no dependent pivot on either side: the refined GPU solution has a KKT
        residual within 100x of the oracle's (or below 1e-9 of the right-hand
        side scale), and while eps_diag is still at its initial 1e-14 the two
        solutions agree to 1e-6 relative;
      * the dependent-pivot classification (ndep, live mask): where the
        oracle's own three summation orders agree on it (every state without
        dependent pivots), the GPU's is identical; where they do not (every
        captured state with dependent pivots: e.g. 25fv47_85 gives 18 / 15 /
        74, afiro_30 3 / 4 / 8, dfl001_114 8 / 32 / 139 -- the reference
        tests d == 0 exactly, ldlt.c:600, on a numerically singular system)
        the classification is not a property of the algorithm, and the GPU
        must recognise the singularity (some dependent pivot) and return
        finite values; the IPM-level tests judge the outcome;
      * pivot by pivot (every pivot live on the GPU and under all three
        orders): the GPU's relative distance from the oracle's pivots, at
        its 99th percentile and at its maximum, within twice the oracle's
        own spread between its orders (floor 1e-9) -- late-iteration
        systems are ill-conditioned enough that a reordered sum moves a
        pivot by 1e-3 (dfl001_100) to O(1) (dfl001_110) under the
        reference's own algorithm, so no fixed tolerance is right for all;
      * the refined solutions (no dependent pivot anywhere, eps_diag still
        1e-14): within max(1e-6 relative, twice the oracle orders' spread).
    Measured on the GPU (tools/kkt_state_compare.py, round 4): the GPU's
    pivot distance is below the orders' spread on every state, e.g.
    dfl001_100 p99 1.1e-3 against 2.9e-3, dfl001_40 max 2.6e-9 against 3.4e-9."""
    name, it = state.rsplit("_", 1)
    st = np.load(os.path.join(GOLDEN, "..", "kkt_states", state + ".npz"))
    E, D, eps = st["E"], st["D"], float(st["epsdiag"])
    p = ipo_amd.load_mps(mps_path(name))
    rng = np.random.default_rng(int(it))
    fy = rng.uniform(-1, 1, p.m)
    fx = rng.uniform(-1, 1, p.n)
    gpu = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
    orc = oracle_lib.OracleKkt(p)
    gpu.set_epsdiag(eps)
    orc.set_epsdiag(eps)
    gpu.factor(E, D)
    orc.factor(E, D)
    gi, oi = gpu.info(), orc.info()
    _, glive = gpu.pivots()
    var = oracle_variants(p, E, D, eps, fy, fx)
    robust = all(np.array_equal(v[1], var[0][1]) for v in var)
    gd = gpu.pivots()[0]
    both = glive.astype(bool) & var[0][1].astype(bool) & var[1][1].astype(bool) & var[2][1].astype(bool)
    rg = _rel(gd[both], var[0][2][both])
    rv = np.maximum(_rel(var[1][2][both], var[0][2][both]), _rel(var[2][2][both], var[0][2][both]))
    if both.any():
        for qq in (0.99, 1.0):
            assert np.quantile(rg, qq) <= max(1e-9, 2 * np.quantile(rv, qq)), (qq, np.quantile(rg, qq),
                                                                                 np.quantile(rv, qq))
    gy, gx, _ = gpu.solve(E, D, fy, fx)
    oy, ox, _ = orc.solve(E, D, fy, fx)
    bc = max(np.abs(fy).max(), np.abs(fx).max()) + 1
    rg = kkt_residual(p, E, D, fy, fx, gy, gx)
    ro = kkt_residual(p, E, D, fy, fx, oy, ox)
    print(f"{state}: ndep gpu {gi['ndep']} oracle {oi['ndep']} eps {gi['epsdiag']:.1e}/{oi['epsdiag']:.1e} "
          f"resid gpu {rg:.3e} oracle {ro:.3e}; oracle orders ndep {[v[0] for v in var]}")
    if robust:
        assert gi["ndep"] == oi["ndep"] and np.array_equal(glive, var[0][1])
    if oi["ndep"] == 0 and gi["ndep"] == 0:
        assert rg <= max(100 * ro, 1e-9 * bc)
        if eps <= 1e-14 and all(v[0] == 0 for v in var):
            scale = 1.0 + max(np.abs(oy).max(), np.abs(ox).max())
            spread = max(max(np.abs(v[3][0] - oy).max(), np.abs(v[3][1] - ox).max()) for v in var[1:])
            bound = max(1e-6 * scale, 2 * spread)
            assert np.abs(gy - oy).max() <= bound and np.abs(gx - ox).max() <= bound, (bound, spread)
    else:
        assert gi["ndep"] > 0 or oi["ndep"] == 0
        assert np.isfinite(gy).all() and np.isfinite(gx).all()


def test_ldltfac_plugin_abi():
    """ldltfac/forwardbackward with the reference's swapped roles (hsd.c:218,223)."""
    import ctypes as C
    p = ipo_amd.load_mps(mps_path("afiro"))
    kAt, iAt, At = p.transpose()
    rng = np.random.default_rng(3)
    E = rng.uniform(0.5, 2, p.m)
    D = rng.uniform(0.5, 2, p.n)
    fy = rng.uniform(-1, 1, p.m)
    fx = rng.uniform(-1, 1, p.n)
    L = ipo_amd.lib()
    kA, iA, A = p.kA.astype(np.int32), p.iA.astype(np.int32), p.A.copy()
    # hsd.c:218  ldltfac(n, m, kAt, iAt, At, E, D, kA, iA, A, v)
    L.ldltfac(p.n, p.m, kAt.ctypes.data, iAt.ctypes.data, At.ctypes.data, E.ctypes.data, D.ctypes.data,
              kA.ctypes.data, iA.ctypes.data, A.ctypes.data, 1)
    y = fy.copy(); x = fx.copy()
    L.forwardbackward(E.ctypes.data, D.ctypes.data, y.ctypes.data, x.ctypes.data)
    L.inv_clo()
    orc = oracle_lib.OracleKkt(p)
    orc.factor(E, D)
    oy, ox, _ = orc.solve(E, D, fy, fx)
    assert np.allclose(y, oy, rtol=1e-9, atol=1e-10)
    assert np.allclose(x, ox, rtol=1e-9, atol=1e-10)
