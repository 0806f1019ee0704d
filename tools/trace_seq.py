"""One IPM iteration's kernel sequence from a rocprofv3 --kernel-trace run
(developer tool): the dispatches between two consecutive k_tail_run
launches around the middle of the run, with each kernel's duration, its
grid and the idle gap before it, and the time per kernel name over that
iteration.

usage: python3 tools/trace_seq.py <rocprofv3 output dir> [iteration index]
       python3 tools/trace_seq.py <rocprofv3 output dir> idle
  (idle: the device's idle time per iteration, over the union of every
  stream's dispatches, and the kernel pairs around gaps above 15 us)
"""
import csv
import glob
import os
import sys


def short(n):
    return n.replace("(anonymous namespace)::", "").split("(")[0]


def idle(rows, tails):
    import statistics as st
    per, big = [], {}
    for k in range(1, len(tails) - 1):
        a, b = tails[k], tails[k + 1]
        end, t_idle = rows[a][1], 0
        for i in range(a + 1, b + 1):
            s, e = rows[i][0], rows[i][1]
            if s > end:
                t_idle += s - end
                if s - end > 15000:
                    key = short(rows[i - 1][2])[-32:] + " -> " + short(rows[i][2])[-32:]
                    big.setdefault(key, []).append((s - end) / 1e3)
            end = max(end, e)
        per.append((t_idle / 1e3, (rows[b][0] - rows[a][0]) / 1e3))
    print(f"iterations {len(per)}: idle us per iteration median {st.median(x[0] for x in per):.1f}, "
          f"iteration median {st.median(x[1] for x in per):.1f} us")
    for key, v in sorted(big.items(), key=lambda x: -sum(x[1])):
        print(f"  {sum(v) / len(per):7.1f} us/iteration  {len(v):4d} gaps, mean {st.mean(v):8.1f} us  {key}")


def main():
    d = sys.argv[1]
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no kernel_trace.csv under {d}")
    rows = []
    with open(files[0]) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0),
                         int(r.get("Workgroup_Size_X", r.get("Workgroup_Size", 0)) or 0)))
    rows.sort()
    tails = [i for i, r in enumerate(rows) if "k_tail_run" in r[2]]
    if len(tails) < 3:
        sys.exit("fewer than three k_tail_run launches")
    if len(sys.argv) > 2 and sys.argv[2] == "idle":
        idle(rows, tails)
        return
    k = int(sys.argv[2]) if len(sys.argv) > 2 else len(tails) // 2
    a, b = tails[k], tails[k + 1]
    t0 = rows[a][0]
    per = {}
    prev_end = None
    print(f"iteration {k}: {b - a} dispatches, {(rows[b][0] - t0) / 1e3:.1f} us from tail run to tail run")
    for r in rows[a:b]:
        gap = (r[0] - prev_end) / 1e3 if prev_end is not None else 0.0
        dur = (r[1] - r[0]) / 1e3
        name = short(r[2])[:60]
        print(f"{(r[0] - t0) / 1e3:9.1f} {dur:8.2f} gap {gap:6.2f}  wg {r[3] // max(1, r[4]):6d}  {name}")
        prev_end = r[1]
        p = per.setdefault(name, [0, 0.0])
        p[0] += 1
        p[1] += dur
    print("per kernel over the iteration (calls, us):")
    for n, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {t:9.1f} {c:4d}  {n}")


if __name__ == "__main__":
    main()
