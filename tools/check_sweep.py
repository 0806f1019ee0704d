#!/usr/bin/env python3
"""Hold a saved GPU sweep (tools/gpu_recipes.sh sweep: gpurun_out/sweep_<method>/
<name>.<method>.txt) to the parity bar of tests/test_gpu_ipm.py offline --
the test's own check functions on every problem -- and print the failures
(developer tool: a whole-set parity check from one GPU call).
usage: python tools/check_sweep.py [dir=gpurun_out] [hsd] [intpt] [hsdls]"""
import os
import sys
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "linear-programming-vanderbei_amd"))

import oracle_lib  # noqa: E402
import test_gpu_ipm as T  # noqa: E402
from conftest import mps_path  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if a not in ("hsd", "intpt", "hsdls")]
    base = args[0] if args else os.path.join(REPO, "gpurun_out")
    meths = [a for a in sys.argv[1:] if a in ("hsd", "intpt", "hsdls")] or ["hsd", "intpt", "hsdls"]
    bad = 0
    for meth in meths:
        d = os.path.join(base, f"sweep_{meth}")
        names = sorted(f[: -len(f".{meth}.txt")] for f in os.listdir(d) if f.endswith(f".{meth}.txt"))
        for name in names:
            text = open(os.path.join(d, f"{name}.{meth}.txt")).read()
            try:
                if meth == "hsd":
                    T.check_hsd(name, text)
                else:
                    table = T.INTPT if meth == "intpt" else T.HSDLS
                    T.check_oracle_method(meth, name, text, oracle_lib.run_cli(mps_path(name), meth), table)
            except AssertionError:
                bad += 1
                print(f"FAIL {meth} {name}: {traceback.format_exc().strip().splitlines()[-1][:300]}")
        print(f"{meth}: {len(names)} problems checked")
    print(f"{bad} failures")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
