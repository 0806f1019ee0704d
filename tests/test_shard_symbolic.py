"""Host symbolic analysis with the linking rows forced into the dense tail
(block-angular sharding); CPU only.

The forced ordering is the build's own extension of the reference's tiered
minimum degree (kkt_symbolic.cpp); what must hold is exactness of the
symbolic factor it reports.  Checked against a brute-force elimination of
the KKT graph in the same order, and for the property sharding relies on:
columns of different blocks never share a row of L outside the tail.
"""
import numpy as np
import pytest

import ipo_amd


def kkt_adjacency(p):
    T = p.m + p.n
    adj = [set() for _ in range(T)]
    for j in range(p.n):
        for r in p.iA[p.kA[j]:p.kA[j + 1]]:
            adj[r].add(p.m + j)
            adj[p.m + j].add(int(r))
    return adj


def brute_colcounts(p, perm):
    """Column counts of L for the KKT graph eliminated in order perm (new -> old)."""
    T = p.m + p.n
    iperm = np.empty(T, np.int64)
    iperm[perm] = np.arange(T)
    a0 = kkt_adjacency(p)
    adj = [set(int(iperm[v]) for v in a0[int(perm[k])]) for k in range(T)]
    cc = np.zeros(T, np.int64)
    for k in range(T):
        later = {v for v in adj[k] if v > k}
        cc[k] = len(later)
        lst = sorted(later)
        for a in lst:
            adj[a].update(lst)
            adj[a].discard(a)
    return cc


@pytest.mark.parametrize("K,nlink", [(2, 6), (3, 20)])
def test_forced_tail_symbolic_is_exact(K, nlink):
    p = ipo_amd.synth_block_angular(K, 40, 150, 4, 16, nlink, 25)
    s = ipo_amd.symbolic_forced(p.m, p.n, p.kA, p.iA, nlink)
    T = p.m + p.n
    assert s["tail_c0"] == T - nlink
    # linking rows last, natural order
    assert np.array_equal(s["perm"][T - nlink:], np.arange(p.m - nlink, p.m))
    assert sorted(s["perm"]) == list(range(T))
    cc = brute_colcounts(p, s["perm"])
    assert np.array_equal(cc, s["colcount"])
    assert s["lnz"] == cc.sum()


def test_forced_zero_is_reference_ordering():
    p = ipo_amd.synth_random(120, 500, 4, 0)
    a = ipo_amd.symbolic(p.m, p.n, p.kA, p.iA)
    b = ipo_amd.symbolic_forced(p.m, p.n, p.kA, p.iA, 0)
    assert np.array_equal(a["perm"], b["perm"]) and a["lnz"] == b["lnz"]


def test_shard_local_symbolic():
    """Each shard's local LP (its blocks' rows + the linking rows, its
    columns) puts the linking rows last and its symbolic factor is exact."""
    K, mb, nb, l = 4, 40, 150, 8
    p = ipo_amd.synth_block_angular(K, mb, nb, 4, 16, l, 25)
    for nsh in (2, 4):
        for k in range(nsh):
            loc = ipo_amd.shard_block_angular(p, nsh, k)
            assert (loc.m, loc.n) == (K // nsh * mb + l, K // nsh * nb)
            sl = ipo_amd.symbolic_forced(loc.m, loc.n, loc.kA, loc.iA, l)
            assert sl["tail_c0"] == loc.m + loc.n - l
            if k == 0:
                assert np.array_equal(brute_colcounts(loc, sl["perm"]), sl["colcount"])
    with pytest.raises(ipo_amd.IpoHipError):
        ipo_amd.shard_block_angular(p, 3, 0)
