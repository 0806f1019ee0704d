"""Per-dispatch breakdown of a rocprofv3 --kernel-trace CSV (developer tool).

Splits every IPM iteration (one k_assemble_A each) into the sparse levels of
the factorisation, the dense tail of the factorisation (after the last
k_update* launch before the first k_tail_syrk, or from the first k_tail_pr,
up to k_min_abs_partial) and
the rest (solves, vector kernels), and prints per region and kernel the
launches and device time per iteration, plus the summed gaps between
consecutive dispatches.

usage: python tools/trace_breakdown.py <kernel_trace.csv> [--json out.json]"""
import csv
import json
import sys
from collections import defaultdict


def short(name):
    name = name.replace("ipo::(anonymous namespace)::", "").replace("ipo::", "")
    return name.split("(")[0].replace("void ", "").strip()


def load(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r.get("Kernel_Name") or r.get("kernel_name") or r.get("Name")
            s = int(r.get("Start_Timestamp") or r.get("start"))
            e = int(r.get("End_Timestamp") or r.get("end"))
            g = r.get("Grid_Size_X") or r.get("Grid_Size") or "0"
            w = r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or "1"
            rows.append((s, e, short(name), int(g) // max(1, int(w))))
    rows.sort()
    return rows


def main():
    rows = load(sys.argv[1])
    its, cur = [], []
    for r in rows:
        if r[2] == "k_assemble_A" and cur:
            its.append(cur)
            cur = []
        cur.append(r)
    its.append(cur)
    its = [it for it in its if any(r[2] == "k_assemble_A" for r in it)][:-1]   # last one: partial
    acc = defaultdict(lambda: [0, 0.0])
    gaps, span = 0.0, 0.0
    for it in its:
        first_syrk = next((i for i, r in enumerate(it) if r[2] == "k_tail_syrk"), None)
        first_pr = next((i for i, r in enumerate(it) if r[2] == "k_tail_pr"), None)
        t1 = next((i for i, r in enumerate(it) if r[2] == "k_min_abs_partial"), len(it))
        t0 = t1
        if first_pr is not None:                         # look-ahead tail: starts at its first step
            t0 = first_pr
        elif first_syrk is not None:
            t0 = max(i for i in range(first_syrk) if it[i][2].startswith("k_update")) + 1
        for i, (s, e, k, g) in enumerate(it):
            region = "factor-sparse" if i < t0 else ("factor-tail" if i < t1 else "solve+vec")
            a = acc[(region, k)]
            a[0] += 1
            a[1] += (e - s) * 1e-3
        span += (it[-1][1] - it[0][0]) * 1e-3
        gaps += sum(max(0, it[i + 1][0] - it[i][1]) for i in range(len(it) - 1)) * 1e-3
    n = max(1, len(its))
    out = {"iterations": len(its), "us_per_iteration_span": span / n, "gap_us_per_iteration": gaps / n,
           "regions": {}}
    tot = defaultdict(float)
    for (region, k), (c, us) in acc.items():
        out["regions"].setdefault(region, {})[k] = {"launches_per_it": c / n, "us_per_it": us / n,
                                                    "avg_us": us / max(c, 1)}
        tot[region] += us / n
    out["region_us_per_it"] = dict(tot)
    print(f"iterations {len(its)}  span/it {span / n:.0f} us  gaps/it {gaps / n:.0f} us")
    for region, t in tot.items():
        print(f"== {region}: {t:.0f} us/it")
        for k, v in sorted(out["regions"][region].items(), key=lambda kv: -kv[1]["us_per_it"]):
            if v["us_per_it"] >= 5:
                print(f"   {k:28s} {v['launches_per_it']:7.1f} launches  {v['us_per_it']:8.1f} us  avg {v['avg_us']:7.2f}")
    if len(sys.argv) > 3 and sys.argv[2] == "--json":
        with open(sys.argv[3], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
