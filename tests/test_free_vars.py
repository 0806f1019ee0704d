"""Free-variable extension (not in the reference).

The reference aborts on a free column with status 3, "dual unbounded"
(solve.c:79-87): 11 replayable netlib problems end there in the golden
traces, which the default path reproduces (test_frontend.py).  With
free="split" (include/ipo_hip.h IPO_HIP_SPLIT_FREE) free columns are split,
x = x+ - x-, or reflected, x = u - x', before the normalisation, and the
problem goes through the unchanged IPM.  There is no reference trace for
this; the pins are (a) the product's transform equals the oracle's
restatement of it (orc_split_free: same dimensions, and the oracle's HSD on
the product's normal form reproduces the oracle CLI's trajectory to the
last printed digit), and (b) the reference-held netlib optima
(problems/netlib/README.md:40-139), reached within the per-problem bar
below.  A split free column makes the KKT system rank-deficient in the
x+ / x- direction (both grow along the null direction), so HSD stops at
mu < 1e-12 with a wider objective error on some problems than on bounded
ones; the bars are those measured with the oracle and are the product's
contract for the extension.
"""
import json
import os
import re

import pytest

import ipo_amd
import oracle_lib
from conftest import REPO, available_problems, golden_trace, mps_path

OPT = json.load(open(os.path.join(REPO, "tests", "golden", "netlib_optima.json")))["problems"]
FREE = sorted(p for p in available_problems() if golden_trace(p).strip().endswith("dual unbounded"))
LINE = re.compile(r"^\s+(\d+)\s+(\S+)\s+(\S+)\s+(\S+)\s+(\S+)(?:\s+(\S+))?\s*$")

# HSD with split free columns: relative error of the final primal objective
# against the README optimum (oracle measurement), or None: no optimum
# claimed (the run ends at the iteration limit)
HSD_BAR = {"capri": 1e-6, "cycle": 2e-3, "greenbeb": 1e-4, "modszk1": 5e-4, "perold": None, "pilot.ja": 1e-3,
           "pilot.we": 1e-3, "pilot4": 2e-2, "stair": 1e-6, "tuff": 1e-5, "vtp.base": 1e-6}
SLOW = {"cycle", "greenbeb", "perold", "pilot.ja", "pilot.we", "pilot4"}


def rows_status(text):
    rows = [m.groups() for m in (LINE.match(ln) for ln in text.splitlines()) if m]
    return rows, text.strip().splitlines()[-1].strip()


def test_free_inventory():
    assert FREE == sorted(HSD_BAR)


@pytest.mark.parametrize("name", FREE)
def test_split_transform_matches_oracle(name):
    """Same normal form: dims line of the oracle's run, and the oracle's HSD
    on the product's arrays prints what the oracle CLI prints (first 8
    iterations)."""
    path = mps_path(name)
    p = ipo_amd.load_mps(path, free="split")
    text = oracle_lib.run_cli(path, "hsd", free="split") if name not in SLOW else None
    if text is not None:
        assert f"m = {p.m},n = {p.n},nz = {p.nz}\n" in text
    r = oracle_lib.solve_arrays(p, "hsd", max_iter=8)
    assert r["iters"] == 8
    if text is not None:
        rows, _ = rows_status(text)
        assert rows[7][1] == f"{r['final_pobj']:.7e}" and rows[7][3] == f"{r['final_dobj']:.7e}"
    with pytest.raises(ipo_amd.IpoHipError):
        ipo_amd.load_mps(path)              # the default keeps the reference's abort (status 3)


@pytest.mark.parametrize("name", [pytest.param(n, marks=pytest.mark.slow) if n in SLOW else n for n in FREE])
def test_split_oracle_reaches_netlib_optimum(name):
    text = oracle_lib.run_cli(mps_path(name), "hsd", free="split", timeout=1200)
    rows, status = rows_status(text)
    bar = HSD_BAR[name]
    if bar is None:
        assert status == "iteration limit"
        return
    assert status == "optimal solution"
    o = OPT[name]
    target = -o["sense"] * o["optimum"]
    assert abs(float(rows[-1][1]) - target) <= bar * max(1.0, abs(target))
