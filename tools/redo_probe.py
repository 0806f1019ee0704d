import os, sys, time
sys.path.insert(0, "linear-programming-vanderbei_amd"); sys.path.insert(0, "tests")
import ipo_amd
from conftest import mps_path
for name in sys.argv[1:]:
    t = time.time(); r = ipo_amd.run_mps(mps_path(name), "hsd"); dt = time.time() - t
    print(name, "coop", os.environ.get("IPO_HIP_COOP_TAIL"), "time %.3f" % dt, r[0] if isinstance(r, tuple) else r, flush=True)
