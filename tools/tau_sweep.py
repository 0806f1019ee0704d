"""Developer tool: iteration counts of the GPU solver for several zero-pivot
tolerances (IPO_HIP_PIVTOL), hsd on every golden problem and intpt on the
rounding_stability intpt set; JSON lines to stdout.
usage: python tools/tau_sweep.py tau1 [tau2 ...]"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import available_problems, golden_trace, mps_path  # noqa: E402
import oracle_lib  # noqa: E402

EXE = os.path.join(REPO, "linear-programming-vanderbei_amd", "bin", "ipo_hip")
STAB = json.load(open(os.path.join(REPO, "tests", "golden", "rounding_stability.json")))
SKIP = set(os.environ.get("SWEEP_SKIP", "").split(","))


def summary(text):
    rows = [ln for ln in text.splitlines() if ln.strip() and ln.strip().split()[0].isdigit() and len(ln.split()) >= 5]
    lines = text.strip().splitlines()
    return len(rows), (lines[-1].strip() if lines else "")


oracle_lib.build()
ref_intpt = {n: summary(oracle_lib.run_cli(mps_path(n), "intpt")) for n in STAB["intpt"]}
for tau in sys.argv[1:]:
    env = dict(os.environ, IPO_HIP_PIVTOL=tau)
    jobs = [(n, "hsd") for n in available_problems() if n not in SKIP] + [(n, "intpt") for n in STAB["intpt"]]
    for name, meth in jobs:
        try:
            out = subprocess.run([EXE, mps_path(name), meth], capture_output=True, text=True, timeout=120, env=env)
            it, st = summary(out.stdout)
        except subprocess.TimeoutExpired:
            it, st = -1, "timeout"
        ri, rs = summary(golden_trace(name)) if meth == "hsd" else ref_intpt[name]
        print(json.dumps({"tau": tau, "method": meth, "name": name, "iters": it, "status": st, "ref_iters": ri,
                          "ref_status": rs}), flush=True)
