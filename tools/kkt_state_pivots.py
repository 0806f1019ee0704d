#!/usr/bin/env python3
"""GPU pivots of captured KKT states (developer tool): factor each
tests/golden/kkt_states/<state>.npz on the GPU and save its pivots D, live
marks and dependent-pivot count to <outdir>/<state>.gpu.npz, for offline
comparison with the oracle's three summation orders
(tools/kkt_state_compare.py).
usage: python tools/kkt_state_pivots.py <outdir> state ..."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "linear-programming-vanderbei_amd"))
import ipo_amd  # noqa: E402
from conftest import mps_path  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
for state in sys.argv[2:]:
    name, it = state.rsplit("_", 1)
    st = np.load(os.path.join(REPO, "tests", "golden", "kkt_states", state + ".npz"))
    p = ipo_amd.load_mps(mps_path(name))
    k = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
    k.set_epsdiag(float(st["epsdiag"]))
    k.factor(st["E"], st["D"])
    d, live = k.pivots()
    info = k.info()
    np.savez_compressed(os.path.join(out, state + ".gpu.npz"), d=d, live=live, ndep=info["ndep"],
                        epsdiag=info["epsdiag"])
    print(state, "ndep", info["ndep"], "eps", info["epsdiag"], flush=True)
    k.close()
