"""A few HSD iterations of BASELINE configs[4] (block-angular, 8 blocks of
25,000 x 100,000 + 512 linking rows) in one process as bench.py's
block_angular leg runs it at N = 1 (a one-rank ShardContext: the linking
rows forced into the dense tail), for kernel traces and counter passes of
tools/profile_round.sh (developer tool).

usage: python tools/blockang_probe.py [iters] [timing 0|1]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "linear-programming-vanderbei_amd"))
import ipo_amd  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    timing = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    p = ipo_amd.synth_block_angular()
    ctx = ipo_amd.ShardContext(ipo_amd.shard_block_angular(p, 1, 0))
    try:
        t0 = time.perf_counter()
        status, st, _ = ctx.run("hsd", max_iter=iters, timing=bool(timing))
        el = time.perf_counter() - t0
    finally:
        ctx.close()
    out = {"iters": st["iters"], "status": status, "ms_per_iteration": 1e3 * el / max(1, st["iters"]),
           "setup_s": ctx.setup_seconds, "levels": st["nlevels"], "final_mu": st["final_mu"]}
    if timing:
        out["phases"] = {name: {"ms_per_iteration": st["phase_ms"][i] / max(1, st["iters"]),
                                "launches_per_iteration": st["phase_launches"][i] / max(1, st["iters"])}
                         for i, name in enumerate(ipo_amd.PHASES) if st["phase_launches"][i]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
