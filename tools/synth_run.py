"""Developer tool: solve a synthetic LP on the GPU and print timing/plan stats.
usage: python tools/synth_run.py random M N BAND [method] | blockang K MB NB L LNZ [method] [shard]
(shard: the block-angular LP as one shard of a 1-rank ShardContext -- linking rows forced into the tail,
as bench.py's block_angular leg runs it)"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "linear-programming-vanderbei_amd"))
import ipo_amd  # noqa: E402

kind = sys.argv[1]
t0 = time.time()
if kind == "random":
    m, n, band = map(int, sys.argv[2:5])
    method = sys.argv[5] if len(sys.argv) > 5 else "hsd"
    p = ipo_amd.synth_random(m, n, 4, band)
else:
    K, mb, nb, l, lnz = map(int, sys.argv[2:7])
    method = sys.argv[7] if len(sys.argv) > 7 and sys.argv[7] != "shard" else "hsd"
    p = ipo_amd.synth_block_angular(K, mb, nb, 4, 256, l, lnz)
print(f"generated m={p.m} n={p.n} nz={p.nz} in {time.time()-t0:.1f}s", flush=True)
t0 = time.time()
ctx = ipo_amd.Context(p) if "shard" not in sys.argv[2:] else ipo_amd.ShardContext(ipo_amd.shard_block_angular(p, 1, 0))
print(f"setup {ctx.setup_seconds:.1f}s (wall {time.time()-t0:.1f}s)", flush=True)
for timing in (False, True):
    t0 = time.time()
    st, s, _ = ctx.run(method, timing=timing)
    dt = time.time() - t0
    keep = {k: s[k] for k in ("iters", "status", "t_solve_s", "final_mu", "final_pobj", "final_dobj", "lnz", "nsup",
                              "nlevels", "refine_passes", "factor_ms", "solve_ms", "flops_factor")}
    keep["phase_ms"] = dict(zip(ipo_amd.PHASES, s["phase_ms"]))
    keep["phase_launches"] = dict(zip(ipo_amd.PHASES, s["phase_launches"]))
    print(json.dumps({"timing": timing, "wall_s": dt, "it_per_s": s["iters"] / s["t_solve_s"], **keep}), flush=True)
