"""Run the GPU ipo_hip driver over every netlib problem (tests/golden) and
record iterations/status/final objectives next to the golden trace.
Output: JSON lines to stdout.  Developer tool (used for profiles/ reports)."""
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import available_problems, golden_trace, mps_path  # noqa: E402

EXE = os.path.join(REPO, "linear-programming-vanderbei_amd", "bin", "ipo_hip")
SKIP = set(os.environ.get("SWEEP_SKIP", "").split(","))
SAVE = os.environ.get("SWEEP_SAVE")          # directory for the full traces (name.method.txt)
METHOD = os.environ.get("SWEEP_METHOD", "hsd")
ONLY = set(filter(None, os.environ.get("SWEEP_ONLY", "").split(",")))   # a subset of the problems


def iters_and_last(text):
    rows = [ln for ln in text.splitlines() if ln.strip() and ln.strip().split()[0].isdigit() and len(ln.split()) >= 5]
    status = text.strip().splitlines()[-1].strip() if text.strip() else ""
    return len(rows), (rows[-1].split() if rows else None), status


for name in available_problems():
    if name in SKIP or (ONLY and name not in ONLY):
        continue
    t0 = time.time()
    try:
        out = subprocess.run([EXE, mps_path(name), METHOD, "--no-out"], capture_output=True, text=True,
                             timeout=int(os.environ.get("SWEEP_TIMEOUT", "120")))
        text, err = out.stdout, out.stderr
        if SAVE:
            os.makedirs(SAVE, exist_ok=True)
            with open(os.path.join(SAVE, f"{name}.{METHOD}.txt"), "w") as fh:
                fh.write(text)
    except subprocess.TimeoutExpired:
        print(json.dumps({"name": name, "timeout": True}), flush=True)
        continue
    n, last, st = iters_and_last(text)
    gn, glast, gst = iters_and_last(golden_trace(name))
    print(json.dumps({"name": name, "iters": n, "golden_iters": gn, "status": st, "golden_status": gst,
                      "last": last, "golden_last": glast, "wall_s": round(time.time() - t0, 3),
                      "stderr": err.strip().splitlines()[-1] if err.strip() else ""}), flush=True)
