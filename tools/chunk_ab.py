#!/usr/bin/env python3
"""Developer A/B: gather chunk floor (IPO_HIP_MIN_CHUNK) on BASELINE configs[3]
banded and dfl001, first iterations with HIP-event phase timing.
usage: chunk_ab.py <min_chunk> [banded|dfl001]"""
import json
import os
import sys
import time

os.environ["IPO_HIP_MIN_CHUNK"] = sys.argv[1]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "linear-programming-vanderbei_amd"), os.path.join(REPO, "tests")]
import ipo_amd  # noqa: E402
from conftest import mps_path  # noqa: E402

which = sys.argv[2] if len(sys.argv) > 2 else "banded"
p = ipo_amd.synth_random(200000, 1000000, 4, 256) if which == "banded" else ipo_amd.load_mps(mps_path("dfl001"))
ctx = ipo_amd.Context(p)
its = 10 if which == "banded" else 117
ctx.run("hsd", max_iter=its)
t0 = time.perf_counter()
st, s, _ = ctx.run("hsd", max_iter=its)
el = time.perf_counter() - t0
st, s2, _ = ctx.run("hsd", max_iter=its, timing=True)
ctx.close()
print(json.dumps({"min_chunk": int(sys.argv[1]), "which": which, "iters": s["iters"], "ms_per_iter": 1e3 * el / s["iters"],
                  "phase_ms_per_iter": {k: round(v / s2["iters"], 3) for k, v in zip(ipo_amd.PHASES, s2["phase_ms"])}}),
      flush=True)
