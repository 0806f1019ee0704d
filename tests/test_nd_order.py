"""Nested-dissection ordering (kkt_order_nd.cpp; not in the reference) on the
host, CPU only.

The reference orders its KKT matrix by tiered minimum degree, and the
library keeps that order (identical permutation, tests/test_symbolic.py)
below kNdMinNodes = 100,000 KKT nodes -- every netlib problem.  Above it,
nested dissection replaces it (K is quasi-definite: it factors under any
symmetric permutation).  What must hold is exactness of the symbolic factor
built on the new order (checked against a brute-force elimination of the
KKT graph, test_shard_symbolic.brute_colcounts), the relaxed supernodes'
padding (column counts only grow, every padded panel is nested), and the
selection rule.  GPU parity of the solves on this order is in
tests/test_synth.py (small LPs against the oracle, configs[3] / configs[4]
at full size against the optimality certificate)."""
import numpy as np
import pytest

import ipo_amd
from test_shard_symbolic import brute_colcounts


@pytest.fixture
def nd_env(monkeypatch):
    def set_(leaf=32, relax=0.0, order="nd"):
        monkeypatch.setenv("IPO_HIP_ORDER", order)
        monkeypatch.setenv("IPO_HIP_ND_LEAF", str(leaf))
        monkeypatch.setenv("IPO_HIP_ND_RELAX", str(relax))
    return set_


def _sym(p, nforced=0):
    return ipo_amd.symbolic_forced(p.m, p.n, p.kA, p.iA, nforced)


@pytest.mark.parametrize("band", [16, 48])
def test_nd_symbolic_is_exact(nd_env, band):
    nd_env(leaf=24, relax=0.0)
    p = ipo_amd.synth_random(600, 3000, 4, band)
    s = _sym(p)
    T = p.m + p.n
    assert sorted(s["perm"]) == list(range(T))
    cc = brute_colcounts(p, s["perm"])
    assert np.array_equal(cc, s["colcount"])
    assert s["lnz"] == cc.sum()
    # dissected: far fewer levels than the minimum-degree chain of a band
    nd_env(order="md")
    md = _sym(p)
    assert s["nlevels"] < md["nlevels"], (s["nlevels"], md["nlevels"])


def test_nd_relaxed_supernodes_pad_only(nd_env):
    """Relaxed supernodes add explicit zeros only: every column count at
    least the exact one, the order unchanged, fewer supernodes."""
    p = ipo_amd.synth_random(600, 3000, 4, 48)
    nd_env(leaf=64, relax=0.0)
    exact = _sym(p)
    nd_env(leaf=64, relax=0.3)
    rel = _sym(p)
    assert np.array_equal(exact["perm"], rel["perm"])
    assert (rel["colcount"] >= exact["colcount"]).all()
    assert rel["lnz"] <= 1.3 * exact["lnz"] + 1
    assert rel["nsup"] < exact["nsup"]


def test_nd_forced_tail_is_exact(nd_env):
    """Block-angular with the linking rows forced last (the shard path)."""
    nd_env(leaf=24, relax=0.0)
    nlink = 10
    p = ipo_amd.synth_block_angular(3, 60, 240, 4, 16, nlink, 30)
    s = _sym(p, nlink)
    T = p.m + p.n
    assert s["tail_c0"] == T - nlink
    assert np.array_equal(s["perm"][T - nlink:], np.arange(p.m - nlink, p.m))
    cc = brute_colcounts(p, s["perm"])
    assert np.array_equal(cc, s["colcount"])


def test_nd_dense_rows_go_last(nd_env):
    """Unforced block-angular: the linking rows (degree far above the
    rows' mean) leave the dissection and are ordered last, in natural
    order; the symbolic factor stays exact."""
    nd_env(leaf=24, relax=0.0)
    nlink = 8
    p = ipo_amd.synth_block_angular(3, 60, 240, 4, 16, nlink, 400)
    s = _sym(p)
    T = p.m + p.n
    assert np.array_equal(s["perm"][T - nlink:], np.arange(p.m - nlink, p.m))
    cc = brute_colcounts(p, s["perm"])
    assert np.array_equal(cc, s["colcount"])


def test_order_selection_by_size(monkeypatch):
    """auto: the reference's minimum degree below 100,000 KKT nodes (all of
    netlib), nested dissection from there; IPO_HIP_ORDER overrides."""
    monkeypatch.delenv("IPO_HIP_ORDER", raising=False)
    small = ipo_amd.synth_random(300, 1500, 4, 32)
    a = ipo_amd.symbolic(small.m, small.n, small.kA, small.iA)
    monkeypatch.setenv("IPO_HIP_ORDER", "md")
    b = ipo_amd.symbolic(small.m, small.n, small.kA, small.iA)
    assert np.array_equal(a["perm"], b["perm"])
    monkeypatch.delenv("IPO_HIP_ORDER")
    big = ipo_amd.synth_random(20000, 100000, 4, 64)
    c = ipo_amd.symbolic(big.m, big.n, big.kA, big.iA)
    monkeypatch.setenv("IPO_HIP_ORDER", "nd")
    d = ipo_amd.symbolic(big.m, big.n, big.kA, big.iA)
    assert np.array_equal(c["perm"], d["perm"])
    assert c["nlevels"] < 200
