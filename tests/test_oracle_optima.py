"""Pin the oracle's intpt.c and hsdls.c restatements to reference-held data.

intpt.c and hsdls.c have no captured trace in the reference (SURVEY.md
8(c)), so their trajectories cannot be pinned line by line.  What the
reference does hold is the optimum of every netlib problem
(problems/netlib/README.md:40-139, copied to tests/golden/netlib_optima.json
by tools/extract_netlib_optima.py).  Wherever the oracle's run of a method
ends "optimal solution", its last printed primal and dual objectives must
equal that optimum; the reference prints the objective of the normalised
problem max c'x (solve.c:202-205 negates c for MIN), i.e. -sense * optimum.

Tolerance: 1e-5 relative (the README gives 11 digits, the trace prints 8,
and both methods stop at their own criteria -- intpt.c:171 absolute 1e-6,
hsdls.c:131 mu < 1e-12 -- not at a fixed objective accuracy).  Wider bars
are listed per problem with the reason: they are where the reference's own
stopping rule leaves the iterate (its HSD golden trace stops at the same
distance, test_hsd_golden_reaches_optimum below).
"""
import json
import os
import re

import pytest

import oracle_lib
from conftest import REPO, available_problems, golden_trace, mps_path

OPT = json.load(open(os.path.join(REPO, "tests", "golden", "netlib_optima.json")))["problems"]
LINE = re.compile(r"^\s+(\d+)\s+(\S+)\s+(\S+)\s+(\S+)\s+(\S+)(?:\s+(\S+))?\s*$")

# oracle runs longer than a few seconds: IPO_SLOW=1
SLOW = {"bnl2", "d2q06c", "d6cube", "dfl001", "greenbea", "ken-11", "pds-06", "pilot", "pilot87", "nesm", "woodw"}

# (method, problem) -> relative tolerance, where the method's own stop leaves
# the iterate farther from the optimum than 1e-5
WIDE = {
    ("hsd", "dfl001"): (1e-3, "README gives 6 digits ('**'); the golden run stops at dual infeasibility 3.8e+02"),
    ("hsd", "sierra"): (1e-3, "golden run stops at mu < 1e-12 with primal infeasibility 6.8e+03"),
    ("hsd", "share1b"): (1e-3, "golden run stops at mu < 1e-12 with primal infeasibility 1.7e-02"),
    ("hsd", "lotfi"): (5e-5, "golden run stops at primal infeasibility 2.0e-04"),
    ("hsdls", "gfrd-pnc"): (1e-4, "stops at mu < 1e-12 with primal infeasibility 8.2e+02"),
}


def last_line(text):
    rows = [m.groups() for m in (LINE.match(ln) for ln in text.splitlines()) if m]
    status = text.strip().splitlines()[-1].strip() if text.strip() else ""
    return (rows[-1] if rows else None), status


def check(method, name, text):
    row, status = last_line(text)
    if status != "optimal solution" or row is None:
        pytest.skip(f"{method} {name}: {status or 'no output'} (no optimum claimed)")
    o = OPT[name]
    target = -o["sense"] * o["optimum"]
    tol = WIDE.get((method, name), (1e-5, ""))[0]
    for col in (1, 3):
        v = float(row[col])
        assert abs(v - target) <= tol * max(1.0, abs(target)), (method, name, col, v, target)


def _params(method):
    return [pytest.param(n, marks=pytest.mark.slow) if n in SLOW else n
            for n in available_problems() if n in OPT]


@pytest.mark.parametrize("name", _params("intpt"))
def test_oracle_intpt_reaches_netlib_optimum(name):
    check("intpt", name, oracle_lib.run_cli(mps_path(name), "intpt", timeout=1200))


@pytest.mark.parametrize("name", _params("hsdls"))
def test_oracle_hsdls_reaches_netlib_optimum(name):
    check("hsdls", name, oracle_lib.run_cli(mps_path(name), "hsdls", timeout=1200))


@pytest.mark.parametrize("name", [n for n in available_problems() if n in OPT])
def test_hsd_golden_reaches_optimum(name):
    """The reference's own HSD traces against the same table: the sign
    convention and the WIDE bars are the reference's, not the oracle's."""
    check("hsd", name, golden_trace(name))


def test_optima_fixture_inventory():
    # 97 replayable problems, 90 with a numeric optimum in the README table
    have = [n for n in available_problems() if n in OPT]
    assert len(have) >= 85
    assert OPT["afiro"]["optimum"] == -4.6475314286e02 and OPT["afiro"]["line"] == 45
