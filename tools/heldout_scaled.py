#!/usr/bin/env python3
"""Held-out problems for the GPU's zero-pivot rule (developer tool; writes
tests/golden/heldout_scaled.json).

The rule |d| <= tau * sum|terms| with tau = 1e-17 (kkt_device.h) was chosen
on the netlib problems the parity tests grade.  These
problems are not that set: each netlib LP in solver() form with every row of
A and b multiplied by a power of two 2^k, k uniform in {-3..3} (seeded):
exact in floating point, the same optimum x, duals y_i / 2^k, but another
interior-point trajectory (hsd.c starts from all ones), other KKT scalings
and other dependent-pivot events.  For each, the oracle (the reference's
algorithm, oracle/) is run under its three summation orders (lltnum's,
reversed, sorted: orc_set_perturb) and the envelope recorded: statuses,
iterations, final objectives -- and a fourth order, the oracle built with
-ffp-contract=fast -mfma (contracted multiply-adds, the FMA order of
tools/rounding_stability.py).  tests/test_gpu_heldout.py holds the GPU to
that envelope with the rule as shipped.

usage: python tools/heldout_scaled.py [maxdim]"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "linear-programming-vanderbei_amd")]
import ipo_amd  # noqa: E402
import oracle_lib  # noqa: E402
from conftest import available_problems, mps_path  # noqa: E402

SEED = 20251121


def scaled(name):
    """The solver-form LP of `name` with row i of A and b scaled by 2^k_i
    (tests/test_gpu_heldout.py repeats this with the seed from the JSON)."""
    p = ipo_amd.load_mps(mps_path(name))
    rng = np.random.default_rng(SEED + sum(map(ord, name)))
    s = np.ldexp(1.0, rng.integers(-3, 4, p.m))
    p.A = p.A * s[p.iA]
    p.b = p.b * s
    return p


def fma_lib(out="/tmp/orcfma_lib"):
    """The oracle library with contracted multiply-adds (built outside the tree)."""
    flags = "-O2 -std=gnu99 -fPIC -ffp-contract=fast -mfma -Wall -Wno-unused-result"
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), f"OUT={out}", f"CFLAGS={flags}",
                    f"{out}/liborc.so"], check=True)
    return C.CDLL(os.path.join(out, "liborc.so"))


def main():
    maxdim = int(sys.argv[1]) if len(sys.argv) > 1 else 12000
    L = oracle_lib.lib()
    Lf = fma_lib()
    out = {"seed": SEED, "scaling": "row i of A and b times 2^k, k uniform in {-3..3}",
           "orders": ["lltnum (the reference's)", "reversed", "sorted", "fma"], "problems": {}}
    for name in available_problems():
        try:
            dims = ipo_amd.mps_dims(mps_path(name))
        except Exception:  # noqa: BLE001
            continue
        if dims[-1] != 0 or dims[3] + dims[4] > maxdim:   # free variables (status 3) or too large
            continue
        p = scaled(name)
        runs = []
        try:
            for order in (0, 1, 2):
                L.orc_set_perturb(order)
                r = oracle_lib.solve_arrays(p, "hsd")
                runs.append({"status": ipo_amd.STATUS_TEXT[r["status"]], "iters": r["iters"],
                             "pobj": r["final_pobj"], "dobj": r["final_dobj"]})
        finally:
            L.orc_set_perturb(0)
        saved = oracle_lib._lib
        try:
            oracle_lib._lib = Lf
            r = oracle_lib.solve_arrays(p, "hsd")
        finally:
            oracle_lib._lib = saved
        runs.append({"status": ipo_amd.STATUS_TEXT[r["status"]], "iters": r["iters"], "pobj": r["final_pobj"],
                     "dobj": r["final_dobj"], "order": "fma"})
        its = [r["iters"] for r in runs]
        stable = len({r["status"] for r in runs}) == 1 and max(its) - min(its) <= 2
        out["problems"][name] = {"orders": runs, "stable": stable}
        print(name, its, [r["status"] for r in runs], flush=True)
    with open(os.path.join(REPO, "tests", "golden", "heldout_scaled.json"), "w") as fh:
        json.dump(out, fh, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
