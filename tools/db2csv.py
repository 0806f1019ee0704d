"""rocprofv3 SQLite output (run_results.db) -> the kernel-trace CSV columns
tools/trace_breakdown.py reads (developer tool).

usage: python tools/db2csv.py <run_results.db> <out.csv>"""
import csv
import sqlite3
import sys


def main():
    c = sqlite3.connect(sys.argv[1])
    names = {r[0]: r[1] for r in c.execute("select id, display_name from rocpd_info_kernel_symbol")}
    rows = c.execute("select kernel_id, start, end, grid_size_x, workgroup_size_x from rocpd_kernel_dispatch order by start")
    with open(sys.argv[2], "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X", "Workgroup_Size_X"])
        for kid, s, e, g, wg in rows:
            w.writerow([names.get(kid, str(kid)), s, e, g, wg])


if __name__ == "__main__":
    main()
