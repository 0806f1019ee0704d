"""Native front end (lp_io.cpp: MPS reader + solvelp transform) against the
golden dimension lines and against the oracle's restatement."""
import re

import numpy as np
import pytest

import ipo_amd
from conftest import available_problems, golden_trace, mps_path


def golden_dims(name):
    t = golden_trace(name)
    pre = re.search(r"m = (\d+),n = (\d+),nz = (\d+) \n", t)
    post = re.search(r"m = (\d+),n = (\d+),nz = (\d+)\n", t)
    return tuple(map(int, pre.groups())), (tuple(map(int, post.groups())) if post else None)


@pytest.mark.parametrize("name", available_problems())
def test_dims_match_golden(name):
    m0, n0, nz0, m, n, nz, st = ipo_amd.mps_dims(mps_path(name))
    pre, post = golden_dims(name)
    assert (m0, n0, nz0) == pre
    if post is None:            # free variable -> "dual unbounded" before solver() (solve.c:79-87)
        assert st == 3
        assert "dual unbounded" in golden_trace(name)
    else:
        assert st == 0
        assert (m, n, nz) == post


@pytest.mark.parametrize("name", ["afiro", "adlittle", "blend", "sc50a", "kb2", "boeing1", "25fv47", "bore3d"])
def test_solver_form_is_well_formed(name):
    p = ipo_amd.load_mps(mps_path(name))
    assert p.kA[0] == 0 and p.kA[-1] == p.nz == len(p.iA) == len(p.A)
    assert np.all(np.diff(p.kA) >= 0)
    for j in range(p.n):          # rows ascend inside each column (solve.c:189)
        col = p.iA[p.kA[j]:p.kA[j + 1]]
        assert np.all(np.diff(col) > 0)
    assert p.iA.min() >= 0 and p.iA.max() < p.m


# writesol (iolp.c:976-1045): the product's report (lp_io.cpp write_sol)
# against the oracle's restatement (orc_writesol) from the same solver()-form
# vectors -- the oracle's own HSD solution -- byte for byte.  The reference
# holds no .out file, so this pins the writer to the oracle only (parity
# unpinned against the reference itself); z is the solver's z in both (the
# reference frees it before writesol reads it, hsd.c:290-291).
WRITESOL = ["afiro", "adlittle", "boeing1", "bore3d", "e226", "fit1d", "kb2", "sc50a", "scorpion", "stocfor1"]


@pytest.mark.parametrize("name", WRITESOL)
def test_writesol_matches_oracle(name, tmp_path):
    import oracle_lib
    path = mps_path(name)
    p = ipo_amd.load_mps(path)
    r = oracle_lib.solve_arrays(p, "hsd")
    a, b = str(tmp_path / "prod.out"), str(tmp_path / "orc.out")
    ipo_amd.write_sol(path, r["x"], r["y"], r["z"], a)
    assert oracle_lib.write_sol(path, r["x"], r["y"], r["z"], b) == 0
    ta, tb = open(a).read(), open(b).read()
    assert ta == tb
    lines = ta.splitlines()
    assert lines[0] == "COLUMNS SECTION" and lines[-1] == "ENDOUT"
    m0, n0 = ipo_amd.mps_dims(path)[:2]
    assert len(lines) == n0 + m0 + 5
