#!/usr/bin/env python3
"""Last printed iteration line of the reference's rounding variants (adds
"<variant>_last" = [iteration, pobj, dobj, mu] to every entry of
tests/golden/rounding_stability.json).

The variants are the reference's own algorithm under other evaluation
orders of its arithmetic (tools/rounding_stability.py: contracted
multiply-adds; tools/order_stability.py: lltnum's sums reversed / by
increasing column).  Their spread of final objectives is the reference's
own rounding envelope on the problems whose iteration count moves under a
rounding change; tests/test_gpu_ipm.py holds the GPU's final objectives to
[min, max] of the base run and its variants, widened by 1e-6 relative,
instead of a flat tolerance.  hsd: the base is the golden trace (the oracle
reproduces all of them byte for byte), intpt / hsdls: the unperturbed oracle.
mu is None for intpt (intpt.c prints none).

usage: python tools/final_lines.py [-j 6] [hsd] [intpt] [hsdls]
"""
import argparse
import concurrent.futures as cf
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
from conftest import golden_trace, mps_path  # noqa: E402
from parting_lines import LINE, PLAIN  # noqa: E402
from rounding_stability import build_fma  # noqa: E402


def last_line(text):
    last = None
    for ln in text.splitlines():
        m = LINE.match(ln)
        if m:
            last = [int(m.group(1)), float(m.group(2)), float(m.group(4)),
                    float(m.group(6)) if m.group(6) is not None else None]
    return last


def run(exe, name, meth, perturb=None):
    env = dict(os.environ)
    if perturb:
        env["ORC_PERTURB"] = perturb
    return subprocess.run([exe, mps_path(name), meth], capture_output=True, text=True, env=env).stdout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=6)
    ap.add_argument("methods", nargs="*", default=["hsd", "intpt", "hsdls"])
    args = ap.parse_args()
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    fma = build_fma("/tmp/orcfma")
    dst = os.path.join(REPO, "tests", "golden", "rounding_stability.json")
    d = json.load(open(dst))
    table = {"intpt": "intpt", "hsdls": "hsdls", "hsd": "problems"}

    def one(job):
        meth, name, var = job
        if var == "golden":
            return job, last_line(golden_trace(name))
        if var == "oracle":
            return job, last_line(run(PLAIN, name, meth))
        if var == "fma":
            return job, last_line(run(fma, name, meth))
        return job, last_line(run(PLAIN, name, meth, var))

    jobs = []
    for meth in args.methods:
        base = "golden" if meth == "hsd" else "oracle"
        for name in d[table[meth]]:
            for var in (base, "fma", "reverse", "sorted"):
                jobs.append((meth, name, var))
    # the long runs first (dfl001, pds-06, ken-13 ... take minutes each)
    slow = ("dfl001", "pds-06", "ken-13", "osa-60", "pilot87", "d2q06c", "cre-d", "cre-b", "fit2p")
    jobs.sort(key=lambda j: (j[1] not in slow, j[1]))
    with cf.ThreadPoolExecutor(args.j) as ex:
        for (meth, name, var), last in ex.map(one, jobs):
            d[table[meth]][name][f"{var}_last"] = last
            print(meth, name, var, last, flush=True)
    d["final_lines"] = ("<variant>_last = [iteration, pobj, dobj, mu] of the last printed line of the base run "
                        "(golden trace / unperturbed oracle) and of each rounding variant (tools/final_lines.py)")
    with open(dst, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
