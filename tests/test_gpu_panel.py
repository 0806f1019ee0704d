"""The fused panel kernels against the per-phase ones: k_diag + k_trsm +
k_tail_syrk (IPO_HIP_PANEL=0, the dependent-pivot path) and the fused
k_panel_s / k_panel_w / look-ahead tail (default) apply the same operations
to every entry of the sparse factor in the same order (the reference's
l = a / d, a -= l (l_j d) form, kkt_dense.hip).  On the dense tail the fused
path defers the trailing update and sums up to four blocks' products in one
accumulator before subtracting them (visits, kkt_dense.hip), so there the two
agree to rounding: refined solves to 1e-10 relative, whole IPM solves to the
HSD parity bar (tests/test_gpu_ipm.py)."""
import os

import numpy as np
import pytest

import ipo_amd
from conftest import mps_path

pytestmark = pytest.mark.gpu

KINDS = ("0", "1")


def _with_panel(kind, fn):
    old = os.environ.get("IPO_HIP_PANEL")
    os.environ["IPO_HIP_PANEL"] = kind
    try:
        return fn()
    finally:
        if old is None:
            del os.environ["IPO_HIP_PANEL"]
        else:
            os.environ["IPO_HIP_PANEL"] = old


@pytest.mark.parametrize("name", ["afiro", "25fv47", "pds-02", "d6cube", "dfl001"])
def test_panel_kinds_solve(name):
    p = ipo_amd.load_mps(mps_path(name))
    rng = np.random.default_rng(7)
    E = rng.uniform(0.1, 10.0, p.m)
    D = rng.uniform(0.1, 10.0, p.n)
    fy = rng.uniform(-1, 1, p.m)
    fx = rng.uniform(-1, 1, p.n)

    def run():
        k = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
        try:
            k.factor(E, D)
            return k.solve(E, D, fy, fx)
        finally:
            k.close()
    outs = [_with_panel(kind, run) for kind in KINDS]
    for gy, gx, ok in outs[1:]:
        assert ok == outs[0][2]
        scale = 1.0 + max(np.abs(outs[0][0]).max(), np.abs(outs[0][1]).max())
        assert np.abs(gy - outs[0][0]).max() <= 1e-10 * scale and np.abs(gx - outs[0][1]).max() <= 1e-10 * scale


@pytest.mark.parametrize("name", ["dfl001"])
def test_panel_kinds_hsd_trace(name):
    """Whole HSD solves (dfl001: 117 iterations, dense tail of 70 block
    columns, dependent-pivot redos) on either path: the golden parity bar."""
    from test_gpu_ipm import check_hsd
    for kind in KINDS:
        check_hsd(name, _with_panel(kind, lambda: ipo_amd.run_mps(mps_path(name), "hsd"))[1])


def _with_env(var, val, fn):
    old = os.environ.get(var)
    os.environ[var] = val
    try:
        return fn()
    finally:
        if old is None:
            del os.environ[var]
        else:
            os.environ[var] = old


def test_sync_free_sweeps_bitwise():
    """The sync-free top-level sweeps (k_fwd_sf / k_bwd_sf) against the
    per-level launches (IPO_HIP_SF=0): the same arithmetic per supernode, so
    the dfl001 HSD traces are identical."""
    texts = [_with_env("IPO_HIP_SF", v, lambda: ipo_amd.run_mps(mps_path("dfl001"), "hsd"))[1] for v in ("0", "1")]
    assert texts[0] == texts[1]


def test_tail_repair():
    """A dependent pivot in the look-ahead dense tail: resuming the look-ahead
    after redoing only the bailed block column (default) and redoing the
    whole factorisation with the per-phase kernels (IPO_HIP_TAIL_REPAIR=0) --
    the dfl001 HSD solve meets such pivots in a few factorisations; both
    solves meet the golden parity bar."""
    from test_gpu_ipm import check_hsd
    for v in ("0", "1"):
        check_hsd("dfl001", _with_env("IPO_HIP_TAIL_REPAIR", v, lambda: ipo_amd.run_mps(mps_path("dfl001"), "hsd"))[1])


def _solve_env(var, val, name="dfl001", extra=()):
    def run():
        return ipo_amd.run_mps(mps_path(name), "hsd")
    fn = run
    for v2, x2 in extra:
        fn = (lambda f, v2=v2, x2=x2: (lambda: _with_env(v2, x2, f)))(fn)
    status, text, st = _with_env(var, val, fn)
    return status, text, {k: st[k] for k in sorted(st) if k.startswith("final") or k == "iters"}


def test_hsd_overlap_bitwise():
    """mu, residuals and right-hand sides on a side stream beside the
    factorisation (default) against the sequential iteration
    (IPO_HIP_OVERLAP=0): the device mu / phi / psi / theta are the host's
    operations in the host's order, so the solves are identical."""
    assert _solve_env("IPO_HIP_OVERLAP", "0") == _solve_env("IPO_HIP_OVERLAP", "1")


def test_tail_chain_pairs_bitwise():
    """Dense-tail substitution chains with two 64-row blocks per workgroup
    (k_tail_fwd_pair / k_tail_bwd_pair, IPO_HIP_CHAIN_PAIRS=1; off by default)
    against one block per workgroup (IPO_HIP_CHAIN_PAIRS=0): the same
    arithmetic in the same order, the first block's z handed on inside the
    workgroup -- identical dfl001 HSD solves (trace and final values).  The
    lead forward sweep is off on both sides (IPO_HIP_CHAIN_LEAD=0), since it
    takes precedence over the forward pair kernel."""
    off = (("IPO_HIP_CHAIN_LEAD", "0"),)
    assert _solve_env("IPO_HIP_CHAIN_PAIRS", "0", extra=off) == _solve_env("IPO_HIP_CHAIN_PAIRS", "1", extra=off)


@pytest.mark.parametrize("name", ["dfl001", "25fv47", "bnl2", "greenbea", "brandy"])
def test_tail_chain_lead_bitwise(name):
    """The forward dense-tail sweep by one lead workgroup with helper
    workgroups (k_tail_fwd_lead, default) against one workgroup per block
    (IPO_HIP_CHAIN_LEAD=0): every lane's partial is the same terms in the
    same order -- identical HSD solves (trace and final values).  Tails of 70
    blocks (dfl001), 7 and 9 (25fv47 nt 396, bnl2 559: odd counts, partial
    last blocks: the extra step after the two-step loop), 12 (greenbea 732,
    partial) and 3 (brandy 155: no helper workgroups)."""
    assert _solve_env("IPO_HIP_CHAIN_LEAD", "0", name) == _solve_env("IPO_HIP_CHAIN_LEAD", "1", name)
