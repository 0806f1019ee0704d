#!/usr/bin/env python3
"""Where the reference's rounding variants part (adds "part_iter" to the
"intpt" and "hsdls" tables of tests/golden/rounding_stability.json).

intpt.c and hsdls.c have no captured trace; the oracle is their reference.
Its three rounding variants (FMA contraction, lltnum sums reversed / sorted:
tools/rounding_stability.py, tools/order_stability.py) are rerun here with
their full traces, and part_iter is the first printed iteration at which any
of them shows a different primal or dual objective from the unperturbed
oracle (more than 1e-6 relative: beyond the 8 printed digits), or the
length of the shorter trace when none does before one ends.  Before that
line the reference's trajectory is a property of its algorithm, not of its
rounding; tests/test_gpu_ipm.py holds the GPU to it line by line there on
the rounding-unstable problems.  hsd.c (argument "hsd") gets the same
column in the "problems" table: where its variants part from the golden
trace.  usage: python tools/parting_lines.py [intpt] [hsdls] [hsd]
"""
import concurrent.futures as cf
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
from conftest import mps_path  # noqa: E402
from rounding_stability import build_fma  # noqa: E402

PLAIN = os.path.join(REPO, "oracle", "build", "ipo_oracle")
LINE = re.compile(r"^\s+(\d+)\s+(\S+)\s+(\S+)\s+(\S+)\s+(\S+)(?:\s+(\S+))?\s*$")


def rows(text):
    return [(float(m.group(2)), float(m.group(4))) for m in (LINE.match(ln) for ln in text.splitlines()) if m]


def trace(exe, name, meth, perturb=None):
    env = dict(os.environ)
    if perturb:
        env["ORC_PERTURB"] = perturb
    return rows(subprocess.run([exe, mps_path(name), meth], capture_output=True, text=True, env=env).stdout)


def rel(a, b):
    return abs(a - b) / max(1.0, abs(b))


def part(base, other):
    for i, (a, b) in enumerate(zip(other, base)):
        if rel(a[0], b[0]) > 1e-6 or rel(a[1], b[1]) > 1e-6:
            return i
    return min(len(base), len(other))


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    fma = build_fma("/tmp/orcfma")
    dst = os.path.join(REPO, "tests", "golden", "rounding_stability.json")
    d = json.load(open(dst))

    def one(job):
        meth, name = job
        base = trace(PLAIN, name, meth)
        others = [trace(fma, name, meth), trace(PLAIN, name, meth, "reverse"), trace(PLAIN, name, meth, "sorted")]
        return job, min(part(base, o) for o in others)

    # hsd's table is d["problems"] (its base trace is the golden one: the
    # oracle reproduces all of them byte for byte)
    table = {"intpt": "intpt", "hsdls": "hsdls", "hsd": "problems"}
    meths = sys.argv[1:] or ["intpt", "hsdls"]
    jobs = [(meth, name) for meth in meths for name in d[table[meth]]]
    with cf.ThreadPoolExecutor(8) as ex:
        for (meth, name), it in ex.map(one, jobs):
            d[table[meth]][name]["part_iter"] = it
    with open(dst, "w") as f:
        json.dump(d, f, indent=1, sort_keys=True)
    for meth in meths:
        t = d[table[meth]]
        print(meth, {n: (v["part_iter"], v.get("oracle_iters", v.get("golden_iters"))) for n, v in sorted(t.items())
                     if not v["stable"]})


if __name__ == "__main__":
    main()
