#!/usr/bin/env python3
"""Exit-time probe under rocprofv3 (developer tool): HSD solves of one
problem, the process's mappings written out (to place a fault address in a
library), then a plain interpreter exit.  Round 3: with the cooperative
dense-tail redo kernel (hipLaunchCooperativeKernel) in the run, the process
faulted at exit inside libhsa-runtime64 (called from libamdhip64's exit
handler) after rocprofv3 had finalised -- also after hipDeviceReset and
with libipo_hip.so unloaded; without that launch it exits 0.
usage: exit_probe.py <mode> [problem] [solves] [maps file]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "linear-programming-vanderbei_amd"), os.path.join(REPO, "tests")]
import ipo_amd  # noqa: E402
from conftest import mps_path  # noqa: E402

name = sys.argv[2] if len(sys.argv) > 2 else "afiro"
for _ in range(int(sys.argv[3]) if len(sys.argv) > 3 else 1):
    status, text, st = ipo_amd.run_mps(mps_path(name), "hsd")
print("status", status, "iters", st["iters"], flush=True)
if len(sys.argv) > 4:      # the process's mappings, to place a fault address in a library
    with open("/proc/self/maps") as src, open(sys.argv[4], "w") as dst:
        dst.write(src.read())
