"""The hbm_roofline leg's kernels alone (bench.py, BASELINE configs[3]
uniform LP), for the rocprofv3 FETCH_SIZE / WRITE_SIZE passes of
tools/profile_round.sh (developer tool).  usage: python tools/hbm_probe.py [reps]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "linear-programming-vanderbei_amd"))
import ipo_amd  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
p = ipo_amd.synth_random(200000, 1000000, 4, 0)
print(json.dumps(ipo_amd.vector_bench(p, reps)), flush=True)
