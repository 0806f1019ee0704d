#!/usr/bin/env python3
"""dfl001 HSD solves with the KKT redo / repair counters printed
(IPO_HIP_DEBUG_REDO), from the package directory given (developer tool:
compares two builds).  usage: redo_stats.py <package dir> [solves]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.abspath(sys.argv[1]), os.path.join(REPO, "tests")]
os.environ["IPO_HIP_DEBUG_REDO"] = "1"
import ipo_amd  # noqa: E402
from conftest import mps_path  # noqa: E402

print("package", ipo_amd.__file__, flush=True)
for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 2):
    t0 = time.perf_counter()
    status, text, st = ipo_amd.run_mps(mps_path("dfl001"), "hsd")
    print("status", status, "iters", st["iters"], "seconds %.3f" % (time.perf_counter() - t0), flush=True)
