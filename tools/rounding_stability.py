"""Classify each netlib problem by whether the reference's iteration count
survives a change of floating-point rounding.

The oracle (oracle/, byte-identical to the reference's captured traces) is
rebuilt with -ffp-contract=fast -mfma, i.e. the same algorithm where every
a*b+c is one rounding instead of two, and rerun on every golden problem.
A problem is "stable" when that perturbed run ends with the same status and
within +-1 iteration of the golden trace; only on stable problems does the
north-star tolerance (iterations within +-1) say anything about an
implementation whose summation order necessarily differs (a GPU
factorisation).  Output: tests/golden/rounding_stability.json.

usage: python tools/rounding_stability.py [--reuse DIR] [-j 8]
  --reuse DIR   parse <name>.mps.out / <name>.out files already produced by
                the FMA oracle in DIR instead of rerunning (dfl001 alone
                takes ~12 min single-threaded).
"""
import argparse
import concurrent.futures as cf
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import available_problems, golden_trace, mps_path  # noqa: E402

ROW = re.compile(r"^\s+(\d+)\s+\S+\s+\S+\s+\S+\s+\S+")


def summarise(text):
    rows = [ln for ln in text.splitlines() if ROW.match(ln)]
    lines = text.strip().splitlines()
    return len(rows), (lines[-1].strip() if lines else "")


def build_fma(out):
    flags = "-O2 -std=gnu99 -fPIC -ffp-contract=fast -mfma -Wall -Wno-unused-result"
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), f"OUT={out}", f"CFLAGS={flags}",
                    f"{out}/ipo_oracle"], check=True)
    return os.path.join(out, "ipo_oracle")


# intpt and hsdls have no published trace: the oracle (contract-off) run is
# the reference there, and the FMA build classifies it the same way.
INTPT_SET = ["afiro", "adlittle", "blend", "sc50a", "sc50b", "kb2", "sc105", "share2b", "stocfor1", "recipe",
             "scagr7", "boeing2", "israel", "bandm", "e226", "ship04s", "25fv47", "capri", "degen2", "agg",
             "scsd1", "fit1d", "brandy", "vtp.base", "lotfi", "beaconfd", "grow7", "sctap1"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reuse")
    ap.add_argument("--out-dir", default="/tmp/orcfma")
    ap.add_argument("-j", type=int, default=8)
    args = ap.parse_args()

    names = available_problems()

    def fma_text(name):
        if args.reuse:
            for f in (f"{name}.mps.out", f"{name}.out"):
                p = os.path.join(args.reuse, f)
                if os.path.exists(p):
                    return open(p).read()
            return None
        r = subprocess.run([exe, mps_path(name)], capture_output=True, text=True)
        return r.stdout

    exe = None if args.reuse else build_fma(args.out_dir)
    with cf.ThreadPoolExecutor(args.j) as ex:
        texts = dict(zip(names, ex.map(fma_text, names)))
    res = {}
    for name in names:
        gi, gs = summarise(golden_trace(name))
        if texts[name] is None:
            continue
        fi, fs = summarise(texts[name])
        res[name] = {"golden_iters": gi, "golden_status": gs, "fma_iters": fi, "fma_status": fs,
                     "stable": fs == gs and abs(fi - gi) <= 1}
    fma_exe = exe or build_fma(args.out_dir)
    plain = os.path.join(REPO, "oracle", "build", "ipo_oracle")
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)

    def other(name, meth):
        a = subprocess.run([plain, mps_path(name), meth], capture_output=True, text=True).stdout
        b = subprocess.run([fma_exe, mps_path(name), meth], capture_output=True, text=True).stdout
        return summarise(a), summarise(b)

    def classify(meth):
        with cf.ThreadPoolExecutor(args.j) as ex:
            r = dict(zip(INTPT_SET, ex.map(lambda n: other(n, meth), INTPT_SET)))
        return {k: {"oracle_iters": a[0], "oracle_status": a[1], "fma_iters": b[0], "fma_status": b[1],
                    "stable": a[1] == b[1] and abs(a[0] - b[0]) <= 1} for k, (a, b) in r.items()}

    ip = classify("intpt")
    hl = classify("hsdls")
    dst = os.path.join(REPO, "tests", "golden", "rounding_stability.json")
    with open(dst, "w") as f:
        json.dump({"method": "oracle rebuilt with -ffp-contract=fast -mfma vs golden traces (hsd) / "
                             "vs the contract-off oracle (intpt, hsdls)",
                   "problems": res, "intpt": ip, "hsdls": hl}, f, indent=1, sort_keys=True)
    ns = sum(v["stable"] for v in res.values())
    print(f"{len(res)} problems, {ns} stable -> {dst}")


if __name__ == "__main__":
    main()
