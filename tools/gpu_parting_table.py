#!/usr/bin/env python3
"""Per-problem table of where the GPU's HSD trace parts from the reference's
captured one (tests/golden/netlib/<name>.mps.sol), from one GPU run of every
replayable netlib problem (developer tool; its output is committed under
profiles/).

For each problem: the GPU's iterations and status next to the golden ones;
"part_line" = the first printed iteration whose primal or dual objective
differs from the golden line by more than 1e-6 relative (beyond the 8
printed digits; the rule tools/parting_lines.py applies to the reference's
own rounding variants), with the golden mu printed on that line; and, from
tests/golden/rounding_stability.json, "variants_part_line" = where the first
of the reference's own rounding variants (FMA contraction, lltnum sums
reversed / sorted) parts from the golden trace.

usage:  python tools/gpu_parting_table.py run <tracedir>        (GPU box: ipo_hip on every problem)
        python tools/gpu_parting_table.py table <tracedir> [out.json]
"""
import json
import os
import re
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import available_problems, golden_trace, mps_path  # noqa: E402

EXE = os.path.join(REPO, "linear-programming-vanderbei_amd", "bin", "ipo_hip")
LINE = re.compile(r"^\s+(\d+)\s+(\S+)\s+(\S+)\s+(\S+)\s+(\S+)(?:\s+(\S+))?\s*$")


def parse(text):
    rows = [tuple(float(v) if v is not None else None for v in m.groups())
            for m in (LINE.match(ln) for ln in text.splitlines()) if m]
    status = text.strip().splitlines()[-1].strip() if text.strip() else ""
    return rows, status


def rel(a, b):
    return abs(a - b) / max(1.0, abs(b))


def run(tdir):
    os.makedirs(tdir, exist_ok=True)
    for name in available_problems():
        t0 = time.time()
        r = subprocess.run([EXE, mps_path(name), "hsd", "--no-out"], capture_output=True, text=True, timeout=300)
        with open(os.path.join(tdir, name + ".hsd.txt"), "w") as fh:
            fh.write(r.stdout)
        print(name, r.returncode, f"{time.time() - t0:.1f}s", flush=True)


def table(tdir, out=None):
    stab = json.load(open(os.path.join(REPO, "tests", "golden", "rounding_stability.json")))["problems"]
    res = {}
    for name in available_problems():
        f = os.path.join(tdir, name + ".hsd.txt")
        if not os.path.exists(f):
            continue
        rows, stat = parse(open(f).read())
        grows, gstat = parse(golden_trace(name))
        part = None
        for i, (r, g) in enumerate(zip(rows, grows)):
            if rel(r[1], g[1]) > 1e-6 or rel(r[3], g[3]) > 1e-6:
                part = i
                break
        if part is None and grows:
            part = min(len(rows), len(grows))
        v = stab.get(name, {})
        res[name] = {"gpu_iters": len(rows), "gpu_status": stat, "golden_iters": len(grows), "golden_status": gstat,
                     "stable": v.get("stable"), "part_line": part,
                     "golden_mu_at_part": grows[part][5] if grows and part is not None and part < len(grows) else None,
                     "variants_part_line": v.get("part_iter")}
    if out:
        with open(out, "w") as fh:
            json.dump({"rule": "first printed iteration whose primal or dual objective differs from the golden "
                               "line by more than 1e-6 relative", "problems": res}, fh, indent=1, sort_keys=True)
    for name, r in sorted(res.items()):
        print(f"{name:10s} gpu {r['gpu_iters']:4d} {r['gpu_status'][:18]:18s} golden {r['golden_iters']:4d} "
              f"{r['golden_status'][:18]:18s} part {r['part_line']} (mu {r['golden_mu_at_part']}) "
              f"variants {r['variants_part_line']} {'stable' if r['stable'] else 'unstable'}")
    return res


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2])
    else:
        table(sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else None)
