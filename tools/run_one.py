#!/usr/bin/env python3
"""Solve one netlib problem on the GPU through ipo_amd.run_mps and print the
trace's last lines and the solve's statistics (developer tool; set IPO_HIP_*
knobs in the environment).  PYTHONPATH may point at another build of the package.
usage: python tools/run_one.py name [method] [repeats]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.append(os.path.join(REPO, "linear-programming-vanderbei_amd"))

import ipo_amd  # noqa: E402
from conftest import mps_path  # noqa: E402


def main():
    name = sys.argv[1]
    meth = sys.argv[2] if len(sys.argv) > 2 else "hsd"
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    print("library:", ipo_amd.LIB_PATH, flush=True)
    for _ in range(reps):
        status, text, st = ipo_amd.run_mps(mps_path(name), meth, timing=True)
        print("\n".join(text.splitlines()[-3:]))
        print(status, {k: st[k] for k in sorted(st) if not isinstance(st[k], (list, dict))}, flush=True)
        if isinstance(st.get("phase_ms"), (list, tuple)) and isinstance(st.get("phase_count"), (list, tuple)):
            print("phases (us per occurrence):", {ph: round(1e3 * ms / max(1, n), 1) for ph, ms, n in
                                                  zip(ipo_amd.PHASES, st["phase_ms"], st["phase_count"]) if n})


if __name__ == "__main__":
    main()
