#!/usr/bin/env python3
"""Compare the GPU's dependent-pivot classification with the oracle's on the
GPU's own factorisation inputs (developer tool, parity investigation).

Input: a directory of IPO_HIP_DUMP_DIR dumps (kkt_device.hip dump_factor)
from a GPU run of one problem.  For every dumped factorisation the oracle
(the reference's lltnum order, ldlt.c:517-636) factors the same K(E, D) with
the same eps_diag; reported per factorisation: ndep on both sides, the
columns whose live mark differs, and their pivots on both sides.

usage: tools/dep_compare.py <problem> <dump dir> [--all]
"""
import glob
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "tests"), os.path.join(REPO, "linear-programming-vanderbei_amd")]
import ipo_amd  # noqa: E402
import oracle_lib  # noqa: E402
from conftest import mps_path  # noqa: E402


def read_dump(path):
    with open(path, "rb") as fh:
        b = fh.read()
    m, n, T, ndep = np.frombuffer(b, np.int32, 4, 0)
    o = 16
    eps_in, eps_out = np.frombuffer(b, np.float64, 2, o); o += 16
    E = np.frombuffer(b, np.float64, m, o); o += 8 * m
    D = np.frombuffer(b, np.float64, n, o); o += 8 * n
    perm = np.frombuffer(b, np.int32, T, o); o += 4 * T
    live = np.frombuffer(b, np.int32, T, o); o += 4 * T
    dg = np.frombuffer(b, np.float64, T, o); o += 8 * T
    dsc = np.frombuffer(b, np.float64, T, o); o += 8 * T
    return dict(m=m, n=n, T=T, ndep=int(ndep), eps_in=eps_in, eps_out=eps_out, E=E, D=D, perm=perm, live=live,
                dg=dg, dscale=dsc)


def main():
    name, ddir = sys.argv[1], sys.argv[2]
    show_all = "--all" in sys.argv
    p = ipo_amd.load_mps(mps_path(name))
    orc = oracle_lib.OracleKkt(p)
    files = sorted(glob.glob(os.path.join(ddir, "f*.bin")))
    first_bad = None
    for i, f in enumerate(files):
        d = read_dump(f)
        assert np.array_equal(d["perm"], orc.perm())
        orc.set_epsdiag(d["eps_in"])
        orc.factor(d["E"], d["D"])
        info = orc.info()
        ol, od = orc.live(), orc.diag()
        diff = np.nonzero(ol != d["live"])[0]
        mark = "" if (len(diff) == 0 and info["ndep"] == d["ndep"]) else "  <-- differs"
        if mark and first_bad is None:
            first_bad = i
        if show_all or mark:
            print(f"factor {i:4d} eps {d['eps_in']:.0e}: ndep gpu {d['ndep']:4d} oracle {info['ndep']:4d}; "
                  f"dropped gpu {int((d['live'] == 0).sum())} oracle {int((ol == 0).sum())}; "
                  f"live marks differ at {len(diff)}{mark}")
            for c in diff[:8]:
                print(f"    col {c} (node {d['perm'][c]}): gpu live {d['live'][c]} d {d['dg'][c]:.6e} "
                      f"|terms| {d['dscale'][c]:.3e}; oracle live {ol[c]} d {od[c]:.6e}")
    print(f"{name}: {len(files)} factorisations, first classification difference at "
          f"{first_bad if first_bad is not None else 'none'}")


if __name__ == "__main__":
    main()
