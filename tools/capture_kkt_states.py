"""Capture realistic KKT scalings (E = w/y, D = z/x, eps_diag) from the CPU
oracle's HSD runs, for the GPU factor/solve parity tests.

Runs oracle/build/ipo_oracle once per problem with ORC_DUMP_ED=<k1,k2,...>
(oracle debug hook that writes the inputs of those factorisations to
/tmp/orc_ed_<k>.bin) and stores them as tests/golden/kkt_states/<problem>_<k>.npz.
Data only; regenerate with
    python tools/capture_kkt_states.py [problem ...]
dfl001's states (late iterations, with and without dependent pivots in the
dense tail) take one ~8 minute oracle run.
"""
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import mps_path  # noqa: E402

CASES = {"afiro": [5, 20, 30], "blend": [10, 25, 27, 29], "share2b": [20, 40], "25fv47": [30, 60, 85],
         "d6cube": [10, 30, 50], "agg2": [20, 50], "degen2": [20, 35], "grow22": [20, 45], "ganges": [30, 50],
         "scfxm2": [40, 70], "israel": [20, 40], "dfl001": [40, 100, 110, 114]}
OUT = os.path.join(REPO, "tests", "golden", "kkt_states")
EXE = os.path.join(REPO, "oracle", "build", "ipo_oracle")


def main():
    os.makedirs(OUT, exist_ok=True)
    only = set(sys.argv[1:])
    for name, iters in CASES.items():
        if only and name not in only:
            continue
        for k in iters:
            if os.path.exists(f"/tmp/orc_ed_{k}.bin"):
                os.unlink(f"/tmp/orc_ed_{k}.bin")
        env = dict(os.environ, ORC_DUMP_ED=",".join(map(str, iters)))
        subprocess.run([EXE, mps_path(name)], env=env, capture_output=True, check=True)
        for k in iters:
            dump = f"/tmp/orc_ed_{k}.bin"
            if not os.path.exists(dump):
                continue
            raw = open(dump, "rb").read()
            m, n = np.frombuffer(raw[:8], np.int32)
            E = np.frombuffer(raw[8:8 + 8 * m], np.float64)
            D = np.frombuffer(raw[8 + 8 * m:8 + 8 * (m + n)], np.float64)
            eps = np.frombuffer(raw[8 + 8 * (m + n):16 + 8 * (m + n)], np.float64)[0]
            np.savez_compressed(os.path.join(OUT, f"{name}_{k}.npz"), E=E, D=D, epsdiag=eps)
            print(name, k, m, n, eps)


if __name__ == "__main__":
    main()
