#!/usr/bin/env python3
"""One line per bench.py log: it/s, ms per iteration, and the per-occurrence
device time of each KKT phase (developer tool).  usage: bench_brief.py log..."""
import json
import sys

for path in sys.argv[1:]:
    line = [ln for ln in open(path) if ln.startswith("{")][-1]
    d = json.loads(line)
    ph = d.get("phases", {})
    parts = " ".join(f"{k} {v['ms_total'] / max(1, v['occurrences']) * 1e3:.0f}" for k, v in ph.items())
    print(f"{path}: {d['value']:.1f} it/s, {d['config'].get('ms_per_iteration', 0):.3f} ms/it, "
          f"iters {d['config'].get('iterations_per_solve', [])[:1]}, phases (us/occurrence): {parts}")
