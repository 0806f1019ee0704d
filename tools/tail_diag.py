#!/usr/bin/env python3
"""Developer diagnostic: factor K(E=1, D=1) of a problem on the GPU with the
factorisation dump on, then compare its pivots with the oracle's column by
column (sparse part vs dense tail).  usage: tools/tail_diag.py outdir name..."""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "linear-programming-vanderbei_amd"),
                os.path.join(REPO, "tools")]
import ipo_amd  # noqa: E402
from conftest import mps_path  # noqa: E402

out = sys.argv[1]
for name in sys.argv[2:]:
    for rho in ("1.0", "0.7"):
        d = os.path.join(out, f"{name}_rho{rho}")
        os.makedirs(d, exist_ok=True)
        code = f"""
import sys, numpy as np
sys.path[:0] = {[os.path.join(REPO, 'tests'), os.path.join(REPO, 'linear-programming-vanderbei_amd')]!r}
import ipo_amd
from conftest import mps_path
p = ipo_amd.load_mps(mps_path({name!r}))
k = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
rng = np.random.default_rng(1)
E = np.ones(p.m); D = np.ones(p.n)
k.factor(E, D)
fy = rng.uniform(-1, 1, p.m); fx = rng.uniform(-1, 1, p.n)
gy, gx, ok = k.solve(E, D, fy, fx)
np.savez({os.path.join(d, 'sol.npz')!r}, gy=gy, gx=gx, fy=fy, fx=fx)
print({name!r}, {rho!r}, k.info())
"""
        env = dict(os.environ, IPO_HIP_DUMP_DIR=d, IPO_HIP_TAIL_DENSITY=rho)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
        print(r.stdout.strip(), r.stderr.strip()[-300:], flush=True)
