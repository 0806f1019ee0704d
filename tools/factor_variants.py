#!/usr/bin/env python3
"""Developer diagnostic: one factorisation of K(E=1, D=1) for a problem under
several kernel-path switches, dumped (IPO_HIP_DUMP_DIR) for comparison with
the oracle (tools/dep_compare.py read_dump).  usage: factor_variants.py
<outdir> <problem> <tail density>.  Round 3 found with it that a level
without windowed-panel units sent the fused launcher into its dense-tail
mode (kkt_dense.hip launch_panel)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
out, name, rho = sys.argv[1], sys.argv[2], sys.argv[3]
variants = {"default": {}, "panel0": {"IPO_HIP_PANEL": "0"}, "repair0": {"IPO_HIP_TAIL_REPAIR": "0"}}
code = f"""
import sys, numpy as np
sys.path[:0] = {[os.path.join(REPO, 'tests'), os.path.join(REPO, 'linear-programming-vanderbei_amd')]!r}
import ipo_amd
from conftest import mps_path
p = ipo_amd.load_mps(mps_path({name!r}))
k = ipo_amd.KktFactor(p.m, p.n, p.kA, p.iA, p.A)
k.factor(np.ones(p.m), np.ones(p.n))
print(k.info())
"""
for v, env in variants.items():
    d = os.path.join(out, f"{name}_{rho}_{v}")
    os.makedirs(d, exist_ok=True)
    e = dict(os.environ, IPO_HIP_DUMP_DIR=d, IPO_HIP_TAIL_DENSITY=rho, IPO_HIP_DEBUG_REDO="1", **env)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=e, timeout=120)
    print(v, r.stdout.strip(), r.stderr.strip()[-400:], flush=True)
