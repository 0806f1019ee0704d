"""The product's host ordering (kkt_symbolic.cpp) must reproduce the
reference's tiered minimum-degree ordering exactly (same permutation, same
L pattern size and op count) -- checked against the oracle restatement."""
import numpy as np
import pytest

import ipo_amd
import oracle_lib
from conftest import mps_path

NAMES = ["afiro", "adlittle", "blend", "sc50a", "sc105", "kb2", "share2b", "israel", "scagr25", "bandm",
         "ship04s", "25fv47", "degen2", "fit1d", "ganges"]


@pytest.mark.parametrize("name", NAMES)
def test_ordering_matches_oracle(name):
    p = ipo_amd.load_mps(mps_path(name))
    mine = ipo_amd.symbolic(p.m, p.n, p.kA, p.iA)
    ok = oracle_lib.OracleKkt(p)
    ref = ok.info()
    assert np.array_equal(mine["perm"], ok.perm())
    assert mine["lnz"] == ref["lnz"]
    assert mine["narth"] == ref["narth"]
    assert mine["denwin"] == ref["denwin"]
    assert mine["pdf"] == ref["pdf"]
    assert mine["nsup"] > 0 and mine["nlevels"] > 0


@pytest.mark.timeout(300)
def test_ordering_matches_oracle_dfl001_threaded(monkeypatch):
    """dfl001 (24,385 nodes): its bit-matrix clique steps reach groups of
    thousands of members, which the product splits over a thread pool
    (kkt_symbolic.cpp StepPool); one thread and eight give the oracle's
    permutation, L size and op count exactly."""
    p = ipo_amd.load_mps(mps_path("dfl001"))
    ok = oracle_lib.OracleKkt(p)
    ref, rperm = ok.info(), ok.perm()
    for threads in ("1", "8"):
        monkeypatch.setenv("IPO_HIP_SETUP_THREADS", threads)
        mine = ipo_amd.symbolic(p.m, p.n, p.kA, p.iA)
        assert np.array_equal(mine["perm"], rperm), threads
        assert (mine["lnz"], mine["narth"], mine["denwin"]) == (ref["lnz"], ref["narth"], ref["denwin"]), threads
