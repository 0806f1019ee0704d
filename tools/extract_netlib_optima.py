#!/usr/bin/env python3
"""Copy the optimum column of the reference's netlib table into a fixture.

Source (data, read as text): /root/reference/problems/netlib/README.md:40-139
("Problem Summary Table", column "Optimal Value").  Output:
tests/golden/netlib_optima.json  {name: {"optimum": float, "digits": int,
"line": README line, "note": str}}.  Entries marked "(see NOTES)" carry no
value and are skipped; dfl001's value is given to 6 digits only ("**").
Also records the objective sense of every available MPS file (MAX / MIN
header keyword, iolp.c:264-353): the reference prints the objective of the
normalised problem  max c'x  (solve.c:202-205 negates c for MIN), so the
printed value is -sense * optimum.

Second fixture, tests/golden/simpo_optima.json: the objective values the
reference's own simplex solver printed for the problems of its evaluation
run (evaluate/v1-cf4d5ba/netlib/simpo/README.md, "Optimal Value"), the only
reference-held optimum of the kennington problems (ken-07, ken-11, ...),
which the netlib table leaves out.  These are printed values (the sign of
the normalised max problem, like ipo's trace), to 8 digits.
"""
import gzip
import json
import os
import re
import sys

REF = "/root/reference/problems/netlib/README.md"
SIMPO = "/root/reference/evaluate/v1-cf4d5ba/netlib/simpo/README.md"
SIMPO_OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                         "simpo_optima.json")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden", "netlib")
OUT = os.path.join(REPO, "tests", "golden", "netlib_optima.json")

ROW = re.compile(r"^\|\s*\[([^\]]+)\]\([^)]*\)\s*\|(.*)\|\s*$")


def sense_of(name):
    path = os.path.join(GOLDEN, name + ".mps.gz")
    if not os.path.exists(path):
        return None
    with gzip.open(path, "rt", errors="replace") as fh:
        for ln in fh:
            w = ln.split()
            if not w:
                continue
            if w[0] == "ROWS":
                return 1
            if w[0] == "MAX":
                return -1
            if w[0] == "MIN":
                return 1
    return 1


def main():
    out = {}
    with open(REF) as fh:
        for lineno, ln in enumerate(fh, 1):
            m = ROW.match(ln)
            if not m:
                continue
            name = m.group(1).lower()
            cells = [c.strip() for c in m.group(2).split("|")]
            opt = cells[-1]
            note = ""
            if "**" in opt:
                note = "README '**': special notation"
                opt = opt.replace("**", "").strip()
            try:
                v = float(opt)
            except ValueError:
                continue
            mant = opt.upper().split("E")[0].replace("-", "").replace(".", "").lstrip("0")
            out[name] = {"optimum": v, "digits": len(mant), "line": lineno, "note": note,
                         "sense": sense_of(name)}
    with open(OUT, "w") as fh:
        json.dump({"source": "problems/netlib/README.md (reference), Optimal Value column",
                   "problems": out}, fh, indent=1, sort_keys=True)
    print(f"{len(out)} optima -> {OUT}", file=sys.stderr)
    simpo = {}
    with open(SIMPO) as fh:
        for lineno, ln in enumerate(fh, 1):
            m = ROW.match(ln)
            if not m:
                continue
            cells = [c.strip() for c in m.group(2).split("|")]
            try:
                simpo[m.group(1).lower()] = {"printed": float(cells[-1]), "line": lineno}
            except ValueError:
                continue
    with open(SIMPO_OUT, "w") as fh:
        json.dump({"source": "evaluate/v1-cf4d5ba/netlib/simpo/README.md (reference), Optimal Value column",
                   "problems": simpo}, fh, indent=1, sort_keys=True)
    print(f"{len(simpo)} simplex optima -> {SIMPO_OUT}", file=sys.stderr)


if __name__ == "__main__":
    main()
