#!/usr/bin/env python3
"""Second stability probe (adds to tests/golden/rounding_stability.json).

tools/rounding_stability.py perturbs the reference's rounding by FMA
contraction only, which keeps lltnum's summation order.  A GPU
factorisation changes that order itself (supernodal MFMA gathers, split-K
partial sums, wave trees), so this probe reruns the oracle (byte-identical
to the reference's traces when unperturbed) with the contributions to each
column summed in two other orders (orc_kkt.c ORC_PERTURB): "reverse" (the
reverse of the reference's linked-list order) and "sorted" (increasing
source column, the order a left-looking supernodal gather visits them).
Same algorithm, same operations; a problem whose iteration count or status
moves under these is chaotic in rounding, and the +-1 iteration bar says
nothing about an implementation with another summation order there.

`stable` becomes: FMA, reverse and sorted all within +-1 of the reference
with its status.  usage: python tools/order_stability.py [-j 8]
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
from conftest import available_problems, golden_trace, mps_path  # noqa: E402
from rounding_stability import INTPT_SET, summarise  # noqa: E402

EXE = os.path.join(REPO, "oracle", "build", "ipo_oracle")
VARIANTS = ("reverse", "sorted")


def run(args):
    name, meth, var = args
    env = dict(os.environ)
    if var:
        env["ORC_PERTURB"] = var
    out = subprocess.run([EXE, mps_path(name), meth], capture_output=True, text=True, env=env).stdout
    return (name, meth, var), summarise(out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-j", type=int, default=8)
    args = ap.parse_args()
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    dst = os.path.join(REPO, "tests", "golden", "rounding_stability.json")
    d = json.load(open(dst))
    jobs = [(n, "hsd", v) for n in d["problems"] for v in VARIANTS]
    for meth in ("intpt", "hsdls"):
        jobs += [(n, meth, v) for n in d[meth] for v in VARIANTS]
    # longest first
    jobs.sort(key=lambda j: -d["problems"].get(j[0], {}).get("golden_iters", 0) * (j[0] in ("dfl001", "pds-06") and 100 or 1))
    with cf.ThreadPoolExecutor(args.j) as ex:
        res = dict(ex.map(run, jobs))
    for name, v in d["problems"].items():
        ok = v["fma_status"] == v["golden_status"] and abs(v["fma_iters"] - v["golden_iters"]) <= 1
        for var in VARIANTS:
            it, st = res[(name, "hsd", var)]
            v[f"{var}_iters"], v[f"{var}_status"] = it, st
            ok = ok and st == v["golden_status"] and abs(it - v["golden_iters"]) <= 1
        v["stable"] = ok
    for meth in ("intpt", "hsdls"):
        for name, v in d[meth].items():
            ok = v["fma_status"] == v["oracle_status"] and abs(v["fma_iters"] - v["oracle_iters"]) <= 1
            for var in VARIANTS:
                it, st = res[(name, meth, var)]
                v[f"{var}_iters"], v[f"{var}_status"] = it, st
                ok = ok and st == v["oracle_status"] and abs(it - v["oracle_iters"]) <= 1
            v["stable"] = ok
    d["method"] = ("oracle rebuilt with -ffp-contract=fast -mfma, and the oracle with lltnum's contributions "
                   "summed in reverse list order / increasing column (ORC_PERTURB), vs golden traces (hsd) / "
                   "vs the unperturbed oracle (intpt, hsdls); stable = all three within +-1 with the same status")
    with open(dst, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    ns = sum(v["stable"] for v in d["problems"].values())
    print(f"{len(d['problems'])} problems, {ns} stable -> {dst}")


if __name__ == "__main__":
    main()
