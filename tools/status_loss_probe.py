"""GPU side of the status-loss study (VERDICT r04 "next" 4; developer tool).

For each problem where the reference ends optimal and the GPU reaches the
200-iteration limit (agg3, maros, d2q06c, share1b), solve it by HSD on the
GPU with IPO_HIP_TRACE_FULL (per iteration: the dependent-pivot count and
eps_diag, ldlt.c:293-306) at the reference's limit, at 2,000 iterations, and
at the reference's limit with eps_diag's growth capped at 1e-6
(IPO_HIP_EPSDIAG_MAX, a diagnostic the library does not use otherwise), and
write one JSON summary: the iteration eps_diag first grows, the
iterations spent at each eps_diag level, the final status / iterations /
mu of both runs.  The oracle side of the same study (oracle/ built with its
ORC_PERTURB summation orders, ORC_DEBUG_STEP per-iteration steps) is in
DESIGN.md section 3.

usage: python tools/status_loss_probe.py out.json [problems...]
"""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBLEMS = ["agg3", "maros", "d2q06c", "share1b"]


def one(name, max_iter):
    """Child process (the trace goes to its stderr): one GPU solve."""
    sys.path.insert(0, os.path.join(REPO, "linear-programming-vanderbei_amd"))
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import ipo_amd
    from conftest import mps_path
    p = ipo_amd.load_mps(mps_path(name))
    r = ipo_amd.solver(p, "hsd", max_iter=max_iter)
    st = r["stats"]
    print(json.dumps({"status": ipo_amd.STATUS_TEXT.get(r["status"], r["status"]), "iters": st["iters"],
                      "final_mu": st["final_mu"], "final_pobj": st["final_pobj"]}), flush=True)


FT = re.compile(r"^FT (\d+) (\S+) (\S+) (\S+) ")
DEP = re.compile(r"^FT\s+ndep=(\d+) eps=(\S+)")


def summarise(stderr):
    eps, ndep, mu = [], [], []
    for ln in stderr.splitlines():
        m = FT.match(ln)
        if m:
            mu.append(float(m.group(4)))
            continue
        m = DEP.match(ln)
        if m:
            ndep.append(int(m.group(1)))
            eps.append(float(m.group(2)))
    levels = {}
    for e in eps:
        levels[f"{e:.0e}"] = levels.get(f"{e:.0e}", 0) + 1
    first_grow = next((i for i, e in enumerate(eps) if e > eps[0]), None) if eps else None
    return {"eps_first_grows_at": first_grow, "iterations_per_eps": levels, "ndep_nonzero_iterations": sum(d > 0 for d in ndep),
            "ndep_first_nonzero_at": next((i for i, d in enumerate(ndep) if d > 0), None),
            "mu_at_eps_1e-5": next((mu[i] for i, e in enumerate(eps) if e >= 1e-5), None) if eps else None,
            "min_mu": min(mu) if mu else None}


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--one":
        one(sys.argv[2], int(sys.argv[3]))
        return
    out = sys.argv[1]
    names = sys.argv[2:] or PROBLEMS
    res = {}
    env = dict(os.environ, IPO_HIP_TRACE_FULL="1")
    for name in names:
        res[name] = {}
        for mi, cap in ((200, None), (2000, None), (200, "1e-6")):
            key = str(mi) + (f"_epsmax{cap}" if cap else "")
            e = dict(env, IPO_HIP_EPSDIAG_MAX=cap) if cap else env
            cp = subprocess.run([sys.executable, __file__, "--one", name, str(mi)], env=e, capture_output=True,
                                text=True, timeout=300)
            if cp.returncode != 0:
                res[name][key] = {"error": cp.stderr[-2000:]}
                print(name, key, "failed", cp.returncode, flush=True)
                break
            r = json.loads(cp.stdout.strip().splitlines()[-1])
            r.update(summarise(cp.stderr))
            res[name][key] = r
            print(name, key, json.dumps(r), flush=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
