"""Kernel-trace CSV (tools/db2csv.py) of a deep-tree factorisation -> per
kernel name: count, mean / median duration, and the idle gap before each
launch (developer tool).  usage: python tools/chain_trace.py <trace.csv>"""
import csv
import statistics
import sys
from collections import defaultdict


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("void ", "").replace("ipo::", "")
    return name.split("(")[0]


def main():
    rows = []
    with open(sys.argv[1]) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                         int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    dur = defaultdict(list)
    gap = defaultdict(list)
    wgs = defaultdict(list)
    prev_end = None
    for s, e, name, g in rows:
        dur[name].append((e - s) / 1e3)
        wgs[name].append(g)
        if prev_end is not None:
            gap[name].append(max(0, s - prev_end) / 1e3)
        prev_end = max(prev_end or 0, e)
    span = (rows[-1][1] - rows[0][0]) / 1e3
    busy = sum(sum(v) for v in dur.values())
    print(f"span {span:.0f} us, kernel time {busy:.0f} us, launches {len(rows)}")
    print(f"{'kernel':60s} {'n':>6s} {'total_ms':>9s} {'mean_us':>8s} {'med_us':>8s} {'gap_us':>7s} {'wg_med':>7s}")
    for name in sorted(dur, key=lambda k: -sum(dur[k])):
        d = dur[name]
        print(f"{name[:60]:60s} {len(d):6d} {sum(d) / 1e3:9.2f} {statistics.mean(d):8.2f} {statistics.median(d):8.2f} "
              f"{statistics.mean(gap[name]) if gap[name] else 0:7.2f} {statistics.median(wgs[name]):7.0f}")
    # the deep chain: gather / panel launches with few workgroups
    for key in ("k_update", "k_panel_w", "k_panel_s"):
        sel = [(e - s) / 1e3 for s, e, n, g in rows if key in n and g <= 64]
        if sel:
            print(f"{key} launches with <= 64 workgroups: {len(sel)}, mean {statistics.mean(sel):.2f} us, "
                  f"median {statistics.median(sel):.2f} us")


if __name__ == "__main__":
    main()
