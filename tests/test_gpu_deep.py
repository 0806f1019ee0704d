"""The deep-tree schedule of the sparse factorisation (kkt_device.hip):
gather slots of finished descendants as "visits" in the launches of lower
levels (on by default from kkt_plan.h kVisitLevels levels up, BASELINE
configs[3]: 2,785 levels), the flat gather kernel (k_update_flat) and the
one-wave leaf sweeps.  Netlib problems are shallow, so the schedule is forced
here (IPO_HIP_VISITS=1, read when a factor object is built) and held to the
same bars as the default schedule: pivots and refined solutions against the
oracle (test_gpu_kkt's tolerances), HSD traces against the golden ones
(test_gpu_ipm.check_hsd).  The flat gather is the pipelined gather's
operations in the same order: bitwise the same factor."""
import contextlib
import os

import numpy as np
import pytest

import ipo_amd
import oracle_lib
from conftest import mps_path
from test_gpu_ipm import STABLE, check_hsd

pytestmark = pytest.mark.gpu

NAMES = ["afiro", "adlittle", "bandm", "ship04s", "25fv47", "degen2", "d6cube", "pds-02"]


@contextlib.contextmanager
def env(**kv):
    old = {k: os.environ.get(k) for k in kv}
    os.environ.update({k: str(v) for k, v in kv.items()})
    try:
        yield
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def system(p, seed=20251121):
    rng = np.random.default_rng(seed)
    return (rng.uniform(0.1, 10.0, p.m), rng.uniform(0.1, 10.0, p.n), rng.uniform(-1, 1, p.m),
            rng.uniform(-1, 1, p.n))


def factor_solve(p, E, D, fy, fx):
    f = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
    try:
        f.factor(E, D)
        gy, gx, ok = f.solve(E, D, fy, fx)
        gd, glive = f.pivots()
        return gy, gx, ok, gd, glive
    finally:
        f.close()


@pytest.mark.parametrize("name", NAMES)
def test_visit_schedule_matches_oracle(name):
    p = ipo_amd.load_mps(mps_path(name))
    E, D, fy, fx = system(p)
    with env(IPO_HIP_VISITS=1):
        gy, gx, ok, gd, glive = factor_solve(p, E, D, fy, fx)
    orc = oracle_lib.OracleKkt(p)
    orc.factor(E, D)
    oy, ox, _ = orc.solve(E, D, fy, fx)
    assert ok == 1
    scale = 1.0 + max(np.abs(oy).max(), np.abs(ox).max())
    assert np.abs(gy - oy).max() <= 1e-8 * scale
    assert np.abs(gx - ox).max() <= 1e-8 * scale
    od = orc.diag()
    assert np.array_equal(glive, orc.live())
    assert (np.abs(gd - od) <= 1e-9 * np.abs(od)).all()


@pytest.mark.parametrize("name", ["afiro", "25fv47", "d6cube", "pds-02"])
def test_flat_gather_bitwise(name):
    """k_update_flat (forced on every small launch, with and without visits)
    gives the pipelined gather's factor bit for bit."""
    p = ipo_amd.load_mps(mps_path(name))
    E, D, fy, fx = system(p)
    for visits in (0, 1):
        with env(IPO_HIP_VISITS=visits, IPO_HIP_GATHER_FLAT=0):
            a = factor_solve(p, E, D, fy, fx)
        with env(IPO_HIP_VISITS=visits, IPO_HIP_GATHER_FLAT=2):
            b = factor_solve(p, E, D, fy, fx)
        for u, v in zip(a, b):
            assert np.array_equal(np.asarray(u), np.asarray(v)), (name, visits)


@pytest.mark.parametrize("name", [n for n in ["afiro", "adlittle", "sc205", "israel", "scfxm2", "ship08s", "sctap1", "agg"]
                                  if n in STABLE])
def test_hsd_trace_with_visit_schedule(name):
    """Whole HSD solves with the deep-tree schedule forced: the golden trace,
    line by line (rounding-stable problems)."""
    with env(IPO_HIP_VISITS=1, IPO_HIP_GATHER_FLAT=1):
        status, text, st = ipo_amd.run_mps(mps_path(name), "hsd")
    check_hsd(name, text)


def test_deep_schedule_envelope_banded():
    """A banded LP whose minimum-degree tree is deep (m 20,000, n 100,000,
    band 256: 468 levels; the order forced to minimum degree, which large LPs
    no longer get by default, kkt_order_nd.cpp), solved with the deep-tree
    schedule (visits and the forward pre-pass k_fwd_pre, on by default at
    this depth) and without it (IPO_HIP_VISITS=0).  The pre-pass subtracts the
    update values from below the narrow range first ((z - pre) - late), so the
    forward sums are not bitwise the level path's: the two solves
    are held to each other at the synthetic LPs' tolerance (same status,
    iterations within +-1, final objectives within 1e-6 relative, HSD's stop
    mu < 1e-12)."""
    p = ipo_amd.synth_random(20000, 100000, 4, 256)
    out = {}
    for visits in (0, 1):
        with env(IPO_HIP_ORDER="md", IPO_HIP_VISITS=visits):
            r = ipo_amd.solver(p, "hsd")
        assert r["stats"]["nlevels"] >= 256
        out[visits] = r
    a, b = out[0], out[1]
    assert a["status"] == b["status"] == 0
    assert abs(a["stats"]["iters"] - b["stats"]["iters"]) <= 1
    for k in ("final_pobj", "final_dobj"):
        assert abs(a["stats"][k] - b["stats"][k]) <= 1e-6 * max(1.0, abs(a["stats"][k]))
    # (status 0 is HSD's stop, mu < 1e-12 in its homogeneous variables,
    # hsd.c:155; stats' final_mu is the last printed iterate's)
