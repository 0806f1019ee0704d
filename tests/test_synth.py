"""Synthetic LPs of BASELINE configs[3] (random sparse) and configs[4]
(block-angular): generator properties on the CPU, the oracle on small
instances, and the GPU path against the oracle (small) and against an
optimality certificate (full size).

The generator is the build's own; the reference has no
synthetic problems, so parity here is against the oracle restatement of
hsd.c (same algorithm) on the same data -- "parity unpinned" by reference
output, pinned by the oracle that reproduces all 97 golden netlib traces.

Tolerances: GPU vs oracle on the same LP: same status, iterations within
+-1, final objectives within 1e-6 relative.  Full-size runs (no oracle in
reasonable time): HSD's own stop (mu < 1e-12, hsd.c:155) plus a KKT
certificate computed here from the returned x, y, w, z:
||Ax + w - b||_inf / (1 + ||b||_inf) <= 1e-6, ||A'y - z - c||_inf /
(1 + ||c||_inf) <= 1e-6, |c'x - b'y| / (1 + |c'x|) <= 1e-6.
"""
import numpy as np
import pytest

import ipo_amd
import oracle_lib


def spmv(p, x):
    cols = np.repeat(np.arange(p.n), np.diff(p.kA))
    return np.bincount(p.iA, weights=p.A * x[cols], minlength=p.m)


def spmv_t(p, y):
    cols = np.repeat(np.arange(p.n), np.diff(p.kA))
    return np.bincount(cols, weights=p.A * y[p.iA], minlength=p.n)


def certificate(p, x, y, w, z):
    pr = np.max(np.abs(spmv(p, x) + w - p.b)) / (1 + np.max(np.abs(p.b)))
    du = np.max(np.abs(spmv_t(p, y) - z - p.c)) / (1 + np.max(np.abs(p.c)))
    cx, by = float(p.c @ x), float(p.b @ y)
    gap = abs(cx - by) / (1 + abs(cx))
    return pr, du, gap


# ---------------------------------------------------------------- CPU: generator
@pytest.mark.parametrize("band", [0, 64])
def test_random_generator_properties(band):
    m, n, k = 500, 2500, 4
    p = ipo_amd.synth_random(m, n, k, band)
    assert p.nz == n * k and np.all(np.diff(p.kA) == k)
    for j in range(n):
        r = p.iA[p.kA[j]:p.kA[j + 1]]
        assert np.all(np.diff(r) > 0) and r[0] >= 0 and r[-1] < m
        if band:
            assert r[-1] - r[0] < band
            centre = j * m // n
            assert r[0] >= max(0, centre - band) and r[-1] < min(m, centre + band)
    a = np.abs(p.A)
    assert a.min() >= 0.1 and a.max() <= 1.0
    for v in (p.xs, p.ys, p.ws, p.zs):
        assert v.min() >= 0.5 and v.max() <= 1.5
    # feasible and bounded by construction (synth.h)
    np.testing.assert_allclose(p.b, spmv(p, p.xs) + p.ws, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(p.c, spmv_t(p, p.ys) - p.zs, rtol=1e-13, atol=1e-13)
    q = ipo_amd.synth_random(m, n, k, band)
    assert np.array_equal(p.iA, q.iA) and np.array_equal(p.A, q.A) and np.array_equal(p.b, q.b)
    r = ipo_amd.synth_random(m, n, k, band, seed=7)
    assert not np.array_equal(p.iA, r.iA)


def test_block_angular_generator_structure():
    K, mb, nb, l, lnz = 3, 200, 800, 16, 150
    p = ipo_amd.synth_block_angular(K, mb, nb, 4, 32, l, lnz)
    assert (p.m, p.n, p.nz) == (K * mb + l, K * nb, K * nb * 4 + l * lnz)
    cols = np.repeat(np.arange(p.n), np.diff(p.kA))
    blk_rows = p.iA < K * mb
    # block columns touch only their own block's rows (and linking rows)
    assert np.array_equal(p.iA[blk_rows] // mb, cols[blk_rows] // nb)
    # every linking row has exactly link_nz entries
    assert np.array_equal(np.bincount(p.iA[~blk_rows] - K * mb, minlength=l), np.full(l, lnz))
    for j in range(p.n):
        assert np.all(np.diff(p.iA[p.kA[j]:p.kA[j + 1]]) > 0)
    np.testing.assert_allclose(p.b, spmv(p, p.xs) + p.ws, rtol=1e-13, atol=1e-13)
    np.testing.assert_allclose(p.c, spmv_t(p, p.ys) - p.zs, rtol=1e-13, atol=1e-13)


def test_generator_rejects_bad_sizes():
    with pytest.raises(ipo_amd.IpoHipError):
        ipo_amd.synth_random(3, 10, 4, 0)


def test_oracle_solves_small_random_lp():
    p = ipo_amd.synth_random(300, 1500, 4, 0)
    r = oracle_lib.solve_arrays(p, "hsd")
    assert r["status"] == 0
    pr, du, gap = certificate(p, r["x"], r["y"], r["w"], r["z"])
    assert pr < 1e-6 and du < 1e-6 and gap < 1e-6


# ---------------------------------------------------------------- GPU
SMALL = [("uniform", dict(m=400, n=2000, per_col=4, band=0)),
         ("banded", dict(m=1000, n=5000, per_col=4, band=64))]


@pytest.mark.gpu
@pytest.mark.parametrize("name,kw", SMALL, ids=[s[0] for s in SMALL])
@pytest.mark.parametrize("method", ["hsd", "intpt"])
def test_gpu_small_synthetic_matches_oracle(name, kw, method):
    p = ipo_amd.synth_random(**kw)
    g = ipo_amd.solver(p, method)
    o = oracle_lib.solve_arrays(p, method)
    assert g["status"] == o["status"] == 0
    assert abs(g["stats"]["iters"] - o["iters"]) <= 1, (g["stats"]["iters"], o["iters"])
    for k in ("final_pobj", "final_dobj"):
        assert abs(g["stats"][k] - o[k]) <= 1e-6 * max(1.0, abs(o[k])), (k, g["stats"][k], o[k])
    pr, du, gap = certificate(p, g["x"], g["y"], g["w"], g["z"])
    assert pr < 1e-6 and du < 1e-6 and gap < 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize("leaf", [16, 1024])
@pytest.mark.parametrize("method", ["hsd", "intpt"])
def test_gpu_nested_dissection_matches_oracle(monkeypatch, method, leaf):
    """The nested-dissection order (kkt_order_nd.cpp, the default from
    100,000 KKT nodes) forced on a small banded LP: the GPU factors K in
    another elimination order than the oracle's minimum degree (the
    reference's), so the solve is the same algorithm in another rounding --
    same status, iterations within +-1, objectives within 1e-6 relative.
    leaf 16: many separators (deep dissection), leaf 1024: one leaf per
    piece of the band."""
    monkeypatch.setenv("IPO_HIP_ORDER", "nd")
    monkeypatch.setenv("IPO_HIP_ND_LEAF", str(leaf))
    p = ipo_amd.synth_random(2000, 10000, 4, 64)
    g = ipo_amd.solver(p, method)
    o = oracle_lib.solve_arrays(p, method)
    assert g["status"] == o["status"] == 0
    assert abs(g["stats"]["iters"] - o["iters"]) <= 1, (g["stats"]["iters"], o["iters"])
    for k in ("final_pobj", "final_dobj"):
        assert abs(g["stats"][k] - o[k]) <= 1e-6 * max(1.0, abs(o[k])), (k, g["stats"][k], o[k])
    pr, du, gap = certificate(p, g["x"], g["y"], g["w"], g["z"])
    assert pr < 1e-6 and du < 1e-6 and gap < 1e-6


@pytest.mark.gpu
def test_gpu_config3_random_banded_full_size():
    """BASELINE configs[3]: m=200k, n=1M, 4 nnz/column, banded (width 256)."""
    p = ipo_amd.synth_random(200_000, 1_000_000, 4, 256)
    g = ipo_amd.solver(p, "hsd")
    assert g["status"] == 0             # HSD stops on mu < 1e-12 (hsd.c:155)
    assert g["stats"]["nlevels"] < 100  # nested dissection (minimum degree: 2,785 levels)
    pr, du, gap = certificate(p, g["x"], g["y"], g["w"], g["z"])
    assert pr < 1e-6 and du < 1e-6 and gap < 1e-6, (pr, du, gap)
