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


@pytest.mark.parametrize("name,method", [("dfl001", "hsd"), ("25fv47", "intpt"), ("greenbea", "hsd")])
def test_level_graph_bitwise(name, method):
    """The sparse levels and the tail gather replayed as one captured HIP
    graph (IPO_HIP_GRAPH=1, opt-in) against the same launches issued one by
    one (default): the same kernels with the same arguments in the same
    order, so the traces are identical."""
    texts = [_with_env("IPO_HIP_GRAPH", v, lambda: ipo_amd.run_mps(mps_path(name), method))[1] for v in ("0", "1")]
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


def test_tail_dependent_pivots_in_panel_bitwise():
    """Dependent pivots of the look-ahead dense tail resolved inside the panel
    launch (IPO_HIP_TAIL_SPEC=1, default: a second panel pass applies the rule
    of ldlt.c:600-614 in the chain, dropped columns checked tile by tile,
    kkt_dense.hip panel_w_body) against the host repair of every such block
    column (IPO_HIP_TAIL_SPEC=0) and against the pass whose every drop is
    taken as contradicted, so that the other workgroups' writes are put back
    (k_tail_restore) before the host repair (IPO_HIP_TAIL_SPEC=2): the same
    operations on every entry, so identical dfl001 HSD solves (trace and final
    values); the in-panel path leaves fewer block columns to the host."""
    runs = {}
    for v in ("0", "1", "2"):
        status, text, st = _with_env("IPO_HIP_TAIL_SPEC", v, lambda: ipo_amd.run_mps(mps_path("dfl001"), "hsd"))
        runs[v] = (status, text, {k: st[k] for k in sorted(st) if k.startswith("final") or k == "iters"},
                   st["tail_repairs"])
    assert runs["0"][:3] == runs["1"][:3] == runs["2"][:3]
    print("tail repairs by the host: spec 0 %d, 1 %d, 2 %d" % (runs["0"][3], runs["1"][3], runs["2"][3]))
    assert runs["0"][3] > 0, "dfl001's HSD solve no longer meets a dependent pivot in the dense tail"
    assert runs["1"][3] < runs["0"][3]
    assert runs["2"][3] >= runs["1"][3]


@pytest.mark.parametrize("var,vals", [("IPO_HIP_TAIL_SPEC", ("0", "1", "2")), ("IPO_HIP_SPARSE_DEP", ("0", "1"))])
@pytest.mark.parametrize("state", ["dfl001_100", "dfl001_110", "dfl001_114"])
def test_tail_dependent_pivots_states_bitwise(state, var, vals):
    """The same three paths on captured late-iteration dfl001 systems
    (tests/golden/kkt_states; many dependent pivots): pivots, live marks and
    the refined solution bit for bit.  Likewise dependent pivots in the
    sparse fused panels resolved in the kernels (IPO_HIP_SPARSE_DEP=1,
    default: exact in k_panel_s, whose wave holds every row of the column; a
    DEP pass in k_panel_w as in the tail, a failed check bailing) against
    the redo of the whole factorisation with the per-phase kernels
    (IPO_HIP_SPARSE_DEP=0)."""
    import os as _os
    st = np.load(_os.path.join(_os.path.dirname(__file__), "golden", "kkt_states", state + ".npz"))
    E, D, eps = st["E"], st["D"], float(st["epsdiag"])
    p = ipo_amd.load_mps(mps_path("dfl001"))
    rng = np.random.default_rng(5)
    fy, fx = rng.uniform(-1, 1, p.m), rng.uniform(-1, 1, p.n)

    def run():
        k = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
        try:
            k.set_epsdiag(eps)
            k.factor(E, D)
            d, live = k.pivots()
            gy, gx, ok = k.solve(E, D, fy, fx)
            return d.copy(), live.copy(), gy, gx, ok, k.info()["ndep"]
        finally:
            k.close()
    outs = [_with_env(var, v, run) for v in vals]
    for o in outs[1:]:
        assert o[4] == outs[0][4] and o[5] == outs[0][5]
        for a, b in zip(o[:4], outs[0][:4]):
            assert np.array_equal(a, b)


@pytest.mark.parametrize("name", ["dfl001", "greenbea"])
def test_tail_visit_schedule_bitwise(name):
    """The look-ahead launches with the capacity-aware visit schedule
    (tail_visit_schedule, default: tiles' first chunks moved into earlier
    launches so that no launch needs more workgroups than the device has
    CUs) against visit_hi's placement alone (IPO_HIP_VISIT_SCHED=0): every
    tile receives the same chunks in the same order, so the HSD solves are
    identical (trace and final values).  The same holds for the launches'
    visit order grouped by XCD (IPO_HIP_VISIT_XCD, default on) against the
    schedule's own order: a launch holds at most one chunk of a tile."""
    assert _solve_env("IPO_HIP_VISIT_SCHED", "0", name) == _solve_env("IPO_HIP_VISIT_SCHED", "1", name)
    assert _solve_env("IPO_HIP_VISIT_XCD", "0", name) == _solve_env("IPO_HIP_VISIT_XCD", "1", name)


@pytest.mark.parametrize("name", ["dfl001", "greenbea", "25fv47"])
def test_tail_run_bitwise(name):
    """The dense tail as one persistent launch (k_tail_run, default: ticketed
    panel and visit items, per-step and per-tile counters) against one launch
    per look-ahead step (IPO_HIP_TAIL_RUN=0), both with the per-step launches'
    visit chunks (the run's latest chunk equal to the chunk, the default
    K = L = 4, pinned here: every tile receives the same chunks of blocks in
    the same order): identical HSD solves (trace and final values) -- the
    hand-offs inside the launch, the window hand-off between steps included,
    deliver what the launch boundaries did."""
    kl = (("IPO_HIP_VISIT_BLOCKS", "4"), ("IPO_HIP_VISIT_LATEST", "4"))
    assert _solve_env("IPO_HIP_TAIL_RUN", "0", name, extra=kl) == _solve_env("IPO_HIP_TAIL_RUN", "1", name, extra=kl)


@pytest.mark.parametrize("name", ["dfl001", "greenbea"])
def test_tail_window_handoff_bitwise(name):
    """The run's window hand-off (RunPub, default: step t + 1's pre-update
    formed window by window from the tile windows step t publishes as they
    complete, the wait for the whole of step t moved after its window chains)
    against the pre-update that waits for step t and reads S
    (IPO_HIP_TAIL_WINPUB=0): the same MFMA k-steps in the same order,
    identical HSD solves."""
    assert _solve_env("IPO_HIP_TAIL_WINPUB", "0", name) == _solve_env("IPO_HIP_TAIL_WINPUB", "1", name)


def test_tail_run_resume_bitwise():
    """The persistent run's bail and resume (IPO_HIP_TAIL_SPEC=0: every
    dependent pivot of the tail goes to the host repair, which resumes the
    run after the bailed block column with its counters kept) against the
    per-step launches' repair: identical dfl001 HSD solves."""
    ext = (("IPO_HIP_VISIT_BLOCKS", "4"), ("IPO_HIP_VISIT_LATEST", "4"), ("IPO_HIP_TAIL_SPEC", "0"))
    a = _solve_env("IPO_HIP_TAIL_RUN", "0", extra=ext)
    b = _solve_env("IPO_HIP_TAIL_RUN", "1", extra=ext)
    assert a == b


def test_sparse_dependent_pivots_bitwise():
    """Whole dfl001 HSD solves with the sparse panels' dependent pivots
    resolved in the kernels (IPO_HIP_SPARSE_DEP=1) and by redoing the
    factorisation (0): identical traces and final values."""
    assert _solve_env("IPO_HIP_SPARSE_DEP", "0") == _solve_env("IPO_HIP_SPARSE_DEP", "1")


def test_small_leaves_bitwise(monkeypatch):
    """Leaf sweeps with the small leaves (<= 8 rows below, <= 8 update-list
    entries) eight to a wave (k_fwd_leaf8 / k_bwd_leaf8), and single-column
    small panels of <= 8 rows factored eight to a wave (k_panel_s1) -- by
    default on levels of >= 32,768 of them, here forced on every level:
    IPO_HIP_SMALL_LEAVES=1 -- against one wave each (IPO_HIP_SMALL_LEAVES=0):
    dfl001 HSD solves identical (trace and final values), and a banded LP
    under nested dissection (10,000 x-node leaves) to the same final
    iterate, bit for bit."""
    assert _solve_env("IPO_HIP_SMALL_LEAVES", "0") == _solve_env("IPO_HIP_SMALL_LEAVES", "1")
    monkeypatch.setenv("IPO_HIP_ORDER", "nd")
    p = ipo_amd.synth_random(2000, 10000, 4, 64)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("IPO_HIP_SMALL_LEAVES", v)
        r = ipo_amd.solver(p, "hsd")
        outs.append((r["status"], r["stats"]["iters"], r["x"], r["y"], r["w"], r["z"]))
    assert outs[0][:2] == outs[1][:2]
    for a, b in zip(outs[0][2:], outs[1][2:]):
        assert np.array_equal(a, b)


def test_split_panel_levels_bitwise(monkeypatch):
    """Wide levels by k_diag + k_trsm instead of the fused panel units (by
    default levels of >= 768 units and >= 4 per supernode; forced on every
    level with >= 4 units per supernode here: IPO_HIP_PANEL_SPLIT=1) against
    the fused units on every level (IPO_HIP_PANEL_SPLIT=0): dfl001 HSD solves
    identical (trace and final values), and a banded LP under nested
    dissection to the same final iterate, bit for bit."""
    assert _solve_env("IPO_HIP_PANEL_SPLIT", "0") == _solve_env("IPO_HIP_PANEL_SPLIT", "1")
    monkeypatch.setenv("IPO_HIP_ORDER", "nd")
    p = ipo_amd.synth_random(2000, 10000, 4, 64)
    outs = []
    for v in ("0", "1"):
        monkeypatch.setenv("IPO_HIP_PANEL_SPLIT", v)
        r = ipo_amd.solver(p, "hsd")
        outs.append((r["status"], r["stats"]["iters"], r["x"], r["y"], r["w"], r["z"]))
    assert outs[0][:2] == outs[1][:2]
    for a, b in zip(outs[0][2:], outs[1][2:]):
        assert np.array_equal(a, b)


def test_merged_level_sweeps_bitwise():
    """A level's leaves and other supernodes in one sweep launch
    (k_fwd_level / k_bwd_level), and a level's fused and small panels in one
    factor launch (k_panel_ws) -- default -- against separate launches
    (IPO_HIP_MERGE_LEVELS=0): the same bodies, so identical dfl001 HSD solves
    (trace and final values)."""
    assert _solve_env("IPO_HIP_MERGE_LEVELS", "0") == _solve_env("IPO_HIP_MERGE_LEVELS", "1")
