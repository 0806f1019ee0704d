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
