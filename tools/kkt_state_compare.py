#!/usr/bin/env python3
"""Compare GPU pivots of captured KKT states (tools/kkt_state_pivots.py) with
the oracle's under its three summation orders (lltnum's, reversed, by source
column: orc_set_perturb).  For every state: ndep and live-mask agreement,
and the relative pivot spread GPU vs oracle against the oracle's own spread
between its orders (quantiles and max over pivots live everywhere).
usage: python tools/kkt_state_compare.py <dir with *.gpu.npz>"""
import glob
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "linear-programming-vanderbei_amd"))
import ipo_amd  # noqa: E402
import oracle_lib  # noqa: E402
from conftest import mps_path  # noqa: E402


def rel(a, b):
    return np.abs(a - b) / np.maximum(np.abs(b), 1e-300)


def main():
    L = oracle_lib.lib()
    out = {}
    for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.gpu.npz"))):
        state = os.path.basename(f)[:-8]
        name, _ = state.rsplit("_", 1)
        g = np.load(f)
        st = np.load(os.path.join(REPO, "tests", "golden", "kkt_states", state + ".npz"))
        p = ipo_amd.load_mps(mps_path(name))
        orc = []
        for order in (0, 1, 2):
            L.orc_set_perturb(order)
            o = oracle_lib.OracleKkt(p)
            o.set_epsdiag(float(st["epsdiag"]))
            o.factor(st["E"], st["D"])
            orc.append((o.info()["ndep"], o.live().copy(), o.diag().copy()))
        L.orc_set_perturb(0)
        live = g["live"].astype(bool) & orc[0][1].astype(bool) & orc[1][1].astype(bool) & orc[2][1].astype(bool)
        rg = rel(g["d"][live], orc[0][2][live])
        rv = np.maximum(rel(orc[1][2][live], orc[0][2][live]), rel(orc[2][2][live], orc[0][2][live]))
        q = lambda a: {k: float(np.quantile(a, v)) for k, v in (("median", 0.5), ("p99", 0.99), ("max", 1.0))}
        out[state] = {"ndep_gpu": int(g["ndep"]), "ndep_oracle_orders": [int(o[0]) for o in orc],
                      "live_equal_oracle": bool(np.array_equal(g["live"], orc[0][1])),
                      "oracle_orders_agree": all(np.array_equal(o[1], orc[0][1]) for o in orc),
                      "pivot_rel_gpu_vs_oracle": q(rg), "pivot_rel_oracle_orders": q(rv)}
        print(state, json.dumps(out[state]), flush=True)
    return out


if __name__ == "__main__":
    main()
