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
    # an "optimal solution" is held to an optimum: where the reference's own
    # order (order 0) ends optimal, as test_gpu_ipm holds it where the golden
    # run does; where it does not, to the published optimum, or else to the
    # objectives of an order that ends optimal (a GPU "optimal"
    # is never passed unchecked).  The one exception is listed with its reason.
    if st == "optimal solution":
        rows, _ = parse(r["trace"])          # the printed last line, as check_optimum reads it
        got = (rows[-1][1], rows[-1][3])
        opt_orders = [o for o in v if o["status"] == "optimal solution"]
        if name in OPT:
            target = -OPT[name]["sense"] * OPT[name]["optimum"]
            tol = WIDE.get(("hsd", name), (1e-5, ""))[0]
            targets = [(target, target)]
        elif opt_orders:
            targets, tol = [(o["pobj"], o["dobj"]) for o in opt_orders], 1e-5
        else:
            targets, tol = [], 0.0
        if v[0]["status"] != "optimal solution" and name in FALSE_OPTIMAL:
            # documented: HSD's mu test ends the solve away from feasibility,
            # where the reference's own order stops at the iteration limit --
            # a status only another order ends with; kept visible as xfail
            assert r["stats"]["final_pinf"] > 1e-6 or r["stats"]["final_dinf"] > 1e-6, (name, FALSE_OPTIMAL[name])
            pytest.xfail(FALSE_OPTIMAL[name])
        assert targets, f"{name}: GPU 'optimal solution' with no optimum to hold it to"
        ok = [all(abs(g - t) <= tol * max(1.0, abs(t)) for g, t in zip(got, tg)) for tg in targets]
        assert any(ok), (name, got, targets, tol)


# Problems whose GPU run may end "optimal solution" by HSD's mu < 1e-12 test
# alone (hsd.c:155) while the iterate is still far from feasible: the
# reference's own order stalls to the iteration limit there, one of the other
# orders stops "optimal" the same way at another objective.  Such an
# "optimal" certifies nothing, so no objective is claimed; the test asserts
# instead that the run is indeed infeasible at its stop.
FALSE_OPTIMAL = {
    "forplan": "scaled forplan: orders 0-2 stop at the iteration limit at objectives 321 / 298 / 165, the FMA order "
               "'optimal' at 522 / 557 with large infeasibilities; the published optimum (-664.2) is reached by none "
               "(the unscaled problem ends the same way on the GPU and under the FMA order, DESIGN.md section 3)",
}
