"""Launch-by-launch timeline of one IPM iteration's factorisation from a
kernel-trace CSV (developer tool).  usage: trace_timeline.py <csv> [iteration] [max_lines]"""
import csv
import sys


def main():
    rows = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r["Kernel_Name"].replace("void ", "").replace("ipo::", "").replace("(anonymous namespace)::", "").split("(")[0]
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name,
                     int(r["Grid_Size_X"]) // max(1, int(r["Workgroup_Size_X"]))))
    rows.sort()
    idx = [i for i, r in enumerate(rows) if r[2].startswith("k_assemble_A")]
    it = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
    lim = int(sys.argv[3]) if len(sys.argv) > 3 else 400
    seg = rows[idx[it]:idx[it + 1]]
    t0 = seg[0][0]
    for s, e, n, g in seg[:lim]:
        print(f"{(s - t0) / 1000:8.1f} {(e - s) / 1000:7.1f}  {n[:28]:28s} {g}")


if __name__ == "__main__":
    main()
