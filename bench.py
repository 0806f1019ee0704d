#!/usr/bin/env python3
"""bench.py -- ipo-hip headline benchmark.

Metric (BASELINE.json): IPM iterations/sec on netlib dfl001, HSD method
(hsd.c, configs[2]), fp64, one MI355X per rank, at the reference's stopping
rule.  A "step" is one complete HSD solve of dfl001 from the reference's
start point to convergence (mu < 1e-12, the metric's "duality gap" proxy,
SURVEY.md 0.6: 117 interior-point iterations, each one KKT assembly +
supernodal LDL' + two refined solves + the O(m+n) step/centering/ratio/
update kernels), with the problem already resident in HBM (setup = upload +
host symbolic analysis, reported apart).  --warmup W untimed solves, then
exactly --steps K timed solves; value = iterations of the K solves / their
wall time.  Every timed solve must end optimal with the golden iteration
count +-1, otherwise value is null and "metric_condition_met" is false: an
unconverged run is not reported under the converged label.

N > 1: dfl001 does not shard, so ranks run independent
replicas; value = all ranks' iterations / max wall time over ranks.

Also reported:
  roofline      -- the dominant phase of the KKT core (most device time in the
                   timed region), measured live with HIP events on the
                   solver's stream; "phases" lists every phase the same way;
  cpu_baseline  -- the CPU oracle (oracle/, a single-threaded restatement of
                   the reference's ipo) timed on this host over a bounded
                   sample of the same workload (rank 0, N = 1);
  hbm_roofline  -- BASELINE configs[3]: the HBM-bound HSD
                   vector kernels timed alone on the uniform random LP
                   (m 200k, n 1M, 4M nonzeros), GB/s against HBM peak;
  block_angular -- BASELINE configs[4]: the synthetic
                   block-angular LP (8 diagonal blocks of 25,000 x 100,000,
                   banded, + 512 linking rows of 2,000 nonzeros) solved by
                   HSD with its blocks sharded over the N ranks, one shard
                   per GPU, RCCL allreduce of the linking-row tail (N = 1:
                   the same algorithm in one process).  Strong scaling (the
                   problem is fixed); not part of `value`.  A watchdog
                   prints the line with this leg marked "timeout" if it
                   does not finish within --ba-timeout seconds.
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "linear-programming-vanderbei_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

METRIC = "IPM iterations/sec (ADA^T factor+solve) on netlib dfl001; duality gap ≤1e-8"
FP64_PEAK_TFLOPS = 78.6    # MI355X FP64 (matrix = vector) dense peak, AMD spec (the guide has no fp64 row)
PHASE_KERNELS = {"gather": "k_update|k_update_flat|k_update_quad",
                 "diag": "k_panel_w|k_panel_s|k_panel_s1|k_panel_ws|k_diag", "trsm": "k_trsm",
                 "tail_syrk": "k_tail_syrk", "tail": "k_tail_run|k_tail_pr|k_tail_col|k_tail_dep|k_tail_restore",
                 "forward": "k_forward|k_fwd_leaf|k_fwd_leaf8|k_fwd_level|k_fwd_diag|k_fwd_gemv|k_fwd_pre|k_fwd_sf|"
                            "k_tail_gather|k_tail_fwd|k_tail_fwd_chain|k_tail_fwd_pair|k_tail_fwd_lead",
                 "backward": "k_backward|k_bwd_leaf|k_bwd_leaf8|k_bwd_level|k_bwd_partial|k_bwd_finish|k_bwd_sf|"
                             "k_tail_dscale|k_tail_bwd|k_tail_bwd_chain|k_tail_bwd_pair"}
HBM_PEAK_GBS = 8000.0      # MI355X HBM3E peak, MI355X_MICROARCH.md
GOLDEN_ITERS = {"dfl001": 117, "25fv47": 91, "afiro": 33}   # evaluate/v1-cf4d5ba/netlib/ipo/*.mps.sol


def dist_env():
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


class Dist:
    """barrier / max / min / sum over ranks and rank 0's bytes everywhere,
    through ipo_amd.hostcomm (TCP star around rank 0; no torch in the
    process, see hostcomm's docstring); a no-op for a single process."""

    def __init__(self):
        from ipo_amd.hostcomm import HostComm
        self.rank, self.world, self.local = dist_env()
        self.comm = HostComm(self.rank, self.world)

    def barrier(self):
        self.comm.barrier()

    def max(self, v):
        return self.comm.reduce_scalar(v, "max")

    def min(self, v):
        return self.comm.reduce_scalar(v, "min")

    def sum(self, v):
        return self.comm.reduce_scalar(v, "sum")

    def bcast_bytes(self, data, n):
        """rank 0's n bytes on every rank"""
        out = self.comm.bcast_bytes(bytes(data) if self.rank == 0 else None)
        assert len(out) == n
        return out

    def close(self):
        self.comm.close()


def timed_replicas(d: Dist, run_step_block, sync):
    """Barrier + sync, run the block, sync + barrier; returns (local result, max seconds over ranks)."""
    sync()
    d.barrier()
    t0 = time.perf_counter()
    res = run_step_block()
    sync()
    d.barrier()
    dt = time.perf_counter() - t0
    return res, d.max(dt)


BA_WORKLOAD = ("synthetic block-angular LP, BASELINE configs[4]: 8 blocks of 25,000 x 100,000 (banded width 256, "
               "4 nnz/column) + 512 linking rows x 2,000 nnz, seed 20251121, hsd")


def block_angular_leg(d, args, sync):
    """BASELINE configs[4] sharded over the ranks; see the module docstring."""
    import ipo_amd
    t0 = time.perf_counter()
    p = ipo_amd.synth_block_angular()                  # configs[4] sizes
    nb = p.blocks["nblocks"]
    if nb % d.world:
        return {"workload": BA_WORKLOAD, "error": f"{nb} blocks do not split over {d.world} ranks"}
    loc = ipo_amd.shard_block_angular(p, d.world, d.rank)
    dims = {"m": p.m, "n": p.n, "nz": p.nz}
    del p
    t_gen = time.perf_counter() - t0
    uid = None
    if d.world > 1:
        uid = d.bcast_bytes(ipo_amd.rccl_unique_id() if d.rank == 0 else None, 128)
    ctx = ipo_amd.ShardContext(loc, d.world, d.rank, rccl_id=uid)
    try:
        if args.ba_warmup > 0:
            ctx.run("hsd", max_iter=args.ba_warmup)
        (status, st, _), el = timed_replicas(d, lambda: ctx.run("hsd", max_iter=args.ba_steps), sync)
        setup = d.max(ctx.setup_seconds)
    finally:
        ctx.close()
    iters = st["iters"]
    # SURVEY.md 8(d)'s per-iteration work of every shard's own factor and
    # solves (the replicated linking-row tail counted on each), summed over
    # the ranks, against N x the per-GPU peak
    fl, by = survey_work(st, loc.m, loc.n, loc.nz)
    fl, by = d.sum(fl), d.sum(by)
    roof = roofline_of(fl / d.world, by / d.world, el / max(iters, 1))
    roof["per"] = "IPM iteration, per GPU (SURVEY.md 8(d) algorithmic work summed over the shards / N)"
    if d.world == 1:
        roof.update(leg_counters("blockang"))
    return {"workload": BA_WORKLOAD, "value": iters / el, "roofline": roof, "unit": "iterations/s", "scaling": "strong",
            "n_gpus": d.world, "parallelism": f"shard{d.world}" if d.world > 1 else "one process",
            "exchange": "RCCL allreduce over xGMI" if d.world > 1 else "none (linking rows in the dense tail)",
            "ms_per_iteration": 1e3 * el / max(iters, 1), "iterations": iters,
            "status": ipo_amd.STATUS_TEXT.get(status, status), "final_mu": st["final_mu"],
            "final_pobj": st["final_pobj"], "final_dobj": st["final_dobj"], **dims,
            "m_local": loc.m, "n_local": loc.n, "nlink": loc.blocks["nlink"], "lnz_local": st["lnz"],
            "setup_s": setup, "generate_s": t_gen}


WATCHDOG_EXIT = 3

BANDED_WORKLOAD = ("synthetic random sparse LP, BASELINE configs[3] banded variant (SURVEY.md 8(d)): m=200,000, "
                   "n=1,000,000, 4 nnz/column in a window of 256 rows around j m / n, seed 20251121, hsd")


def survey_work(st, m, n, nz, solves=2):
    """SURVEY.md 8(d)'s algorithmic work of one IPM iteration (the unit of the
    roofline fraction): flops = narth + s (4 nnz(L) + N) + 2 nz (2 + 2 s),
    bytes = 12 nnz(L) (2 + 2 s) + 12 nz (2 + 2 s) + 8 (m + n) 40, with s the
    solves per iteration (2 for hsd) and N = m + n (the KKT dimension)."""
    N, L = m + n, st["lnz"]
    flops = st["narth"] + solves * (4.0 * L + N) + 2.0 * nz * (2 + 2 * solves)
    byts = 12.0 * L * (2 + 2 * solves) + 12.0 * nz * (2 + 2 * solves) + 8.0 * N * 40
    return flops, byts


def roofline_of(flops, byts, seconds):
    """The binding roofline of a (flops, bytes) workload done in `seconds`."""
    if flops / (FP64_PEAK_TFLOPS * 1e12) >= byts / (HBM_PEAK_GBS * 1e9):
        a = flops / seconds / 1e12
        return {"bound": "mfma", "achieved": a, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": a / FP64_PEAK_TFLOPS,
                "traffic": None, "algorithmic_flops": flops, "algorithmic_bytes": byts}
    a = byts / seconds / 1e9
    return {"bound": "hbm", "achieved": a, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": a / HBM_PEAK_GBS,
            "traffic": None, "algorithmic_flops": flops, "algorithmic_bytes": byts}


def leg_counters(leg):
    """HBM bytes and f64 MFMA flops per IPM iteration of a synthetic leg from
    the newest committed probe profile (profiles/<round>_<leg>_profile.json,
    tools/profile_round.sh + tools/profile_summary.py), or {}."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", f"*_{leg}_profile.json")))
    if not files:
        return {}
    d = json.load(open(files[-1]))
    out = {"traffic_source": os.path.basename(files[-1])}
    if "hbm_bytes_per_iteration" in d:
        out["traffic"] = d["hbm_bytes_per_iteration"]
    if d.get("mfma_util_over_kernel_time") is not None:
        out["mfma_util"] = d["mfma_util_over_kernel_time"]
        out["f64_mfma_flops_per_iteration"] = d.get("f64_mfma_flops_per_iteration")
    return out


def banded_leg(args):
    """BASELINE configs[3], banded variant: the whole HSD solve (factor +
    refined solves every iteration) on one GPU; it/s and the roofline
    fraction of SURVEY.md 8(d)'s per-iteration work.  A second, short run
    (5 iterations, HIP events) splits the time by phase."""
    import ipo_amd
    t0 = time.perf_counter()
    p = ipo_amd.synth_random(200000, 1000000, 4, 256)
    t_gen = time.perf_counter() - t0
    ctx = ipo_amd.Context(p)
    try:
        t0 = time.perf_counter()
        status, st, _ = ctx.run("hsd")
        el = time.perf_counter() - t0
        _, stt, _ = ctx.run("hsd", max_iter=5, timing=True)
    finally:
        ctx.close()
    it = st["iters"]
    flops, byts = survey_work(st, p.m, p.n, p.nz)
    roof = roofline_of(flops, byts, el / max(it, 1))
    roof["per"] = "IPM iteration (SURVEY.md 8(d) algorithmic work)"
    roof.update(leg_counters("banded"))
    ph = {name: {"ms_per_iteration": stt["phase_ms"][i] / 5, "launches_per_iteration": stt["phase_launches"][i] / 5}
          for i, name in enumerate(ipo_amd.PHASES) if stt["phase_launches"][i]}
    return {"workload": BANDED_WORKLOAD, "value": it / el, "unit": "iterations/s", "n_gpus": 1,
            "ms_per_iteration": 1e3 * el / max(it, 1), "iterations": it, "status": ipo_amd.STATUS_TEXT.get(status, status),
            "final_mu": st["final_mu"], "final_pobj": st["final_pobj"], "final_dobj": st["final_dobj"],
            "m": p.m, "n": p.n, "nz": p.nz, "lnz": st["lnz"], "nsup": st["nsup"], "levels": st["nlevels"],
            "refine_passes": st["refine_passes"], "setup_s": ctx.setup_seconds, "generate_s": t_gen,
            "roofline": roof, "phases_first_5_iterations": ph,
            "round1_reference_value": 1.8}


INTPT_WORKLOAD = "netlib 25fv47 by the path-following method (intpt.c:133-238), fp64, BASELINE configs[1], one GPU"


def oracle_run(mps, method, iters=200):
    """The CPU oracle (oracle/, single-threaded C restatement of ipo) on one
    solve of `mps`: (status, iterations, loop seconds, setup seconds)."""
    import oracle_lib

    class Run(C.Structure):
        _fields_ = [("trace", C.c_void_p), ("max_iter", C.c_int), ("iters", C.c_int), ("t_setup", C.c_double),
                    ("t_total", C.c_double), ("final_mu", C.c_double), ("final_pobj", C.c_double),
                    ("final_dobj", C.c_double), ("final_pinf", C.c_double), ("final_dinf", C.c_double)]
    oracle_lib.build()
    L = oracle_lib.lib()
    L.orc_ipo_run.argtypes = [C.c_char_p, C.c_int, C.c_void_p, C.POINTER(Run)]
    L.orc_ipo_run.restype = C.c_int
    r = Run()
    r.max_iter = iters
    st = L.orc_ipo_run(mps.encode(), {"hsd": 0, "intpt": 1, "hsdls": 2}[method], None, C.byref(r))
    return st, r.iters, r.t_total - r.t_setup, r.t_setup


def intpt_leg(args, sync, cpu=None):
    """BASELINE configs[1]: netlib 25fv47 by intpt (intpt.c:133-238; one KKT
    factorisation and one refined solve per iteration) on one GPU, problem
    resident in HBM; a step is one complete solve to intpt's own stop
    (intpt.c:171).  Beside it the CPU oracle's intpt on the same file (one
    thread, whole solves repeated for ~10 s) and SURVEY.md 8(d)'s per-iteration
    roofline (s = 1 solve per iteration)."""
    import ipo_amd
    from conftest import mps_path
    path = mps_path("25fv47")
    p = ipo_amd.load_mps(path)
    ctx = ipo_amd.Context(p)
    try:
        for _ in range(max(1, args.warmup)):
            ctx.run("intpt")
        sync()
        t0 = time.perf_counter()
        runs = [ctx.run("intpt") for _ in range(args.intpt_steps)]
        sync()
        el = time.perf_counter() - t0
        _, stt, _ = ctx.run("intpt", timing=True)
    finally:
        ctx.close()
    status, st, _ = runs[-1]
    iters = sum(r[1]["iters"] for r in runs)
    ok = all(r[0] == 0 for r in runs)
    flops, byts = survey_work(st, p.m, p.n, p.nz, solves=1)
    roof = roofline_of(flops, byts, el / max(iters, 1))
    roof["per"] = "IPM iteration (SURVEY.md 8(d) algorithmic work, s = 1), timed region"
    ph = {name: {"ms_per_solve": stt["phase_ms"][i], "launches_per_solve": stt["phase_launches"][i]}
          for i, name in enumerate(ipo_amd.PHASES) if stt["phase_launches"][i]}
    out = {"workload": INTPT_WORKLOAD, "value": iters / el if ok else None, "unit": "iterations/s", "n_gpus": 1,
           "steps": args.intpt_steps, "ms_per_step": 1e3 * el / max(args.intpt_steps, 1),
           "ms_per_iteration": 1e3 * el / max(iters, 1), "iterations_per_solve": [r[1]["iters"] for r in runs],
           "status": ipo_amd.STATUS_TEXT.get(status, status), "final_pobj": st["final_pobj"],
           "final_dobj": st["final_dobj"], "m": p.m, "n": p.n, "nz": p.nz, "lnz": st["lnz"],
           "setup_s": ctx.setup_seconds, "roofline": roof, "phases_one_solve": ph,
           "published_optimum": 5.5018458883e3}
    if cpu is not None:
        out["cpu_baseline"] = cpu
        if out["value"] is not None and "value" in cpu:
            out["speedup_vs_cpu_baseline"] = out["value"] / cpu["value"]
    return out


def intpt_cpu_baseline():
    """The oracle's intpt on 25fv47 (one thread, whole solves repeated for
    ~10 s), pinned to one core before the GPU is initialised."""
    from conftest import mps_path
    path = mps_path("25fv47")

    def loop():
        t_loop, n_it, n_solves = 0.0, 0, 0
        while t_loop < 10.0 and n_solves < 40:
            cst, ci, cl, _ = oracle_run(path, "intpt")
            t_loop, n_it, n_solves = t_loop + cl, n_it + ci, n_solves + 1
        return t_loop, n_it, n_solves, cst, ci
    (t_loop, n_it, n_solves, cst, ci), core = pinned(loop)
    return {"value": n_it / t_loop, "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": f"{n_solves} complete 25fv47 intpt solves of {ci} iterations (status "
                      f"{cst}), oracle/ C restatement, single thread, symbolic setup excluded, "
                      f"{t_loop:.1f}s timed", "oracle_iterations": ci, "pinned_core": core,
            "cpu_model": host_cpu_model(), "when": "before the GPU is initialised"}


HBM_WORKLOAD = ("synthetic random sparse LP, BASELINE configs[3] uniform variant: m=200,000, n=1,000,000, "
                "4 nnz/column (4.0e6, density 0.002%), seed 20251121")


def hbm_roofline_leg(reps):
    """BASELINE configs[3]: the HBM-bound HSD vector kernels
    (A x / A'y residuals, directions + ratio test, step) timed alone on the
    uniform random LP, device-resident; algorithmic bytes per launch over the
    average launch time against the HBM peak.  The factorisation of this LP
    is not attempted (uniform rows make L near-dense)."""
    import ipo_amd
    p = ipo_amd.synth_random(200000, 1000000, 4, 0)
    res = ipo_amd.vector_bench(p, reps)
    kernels = {}
    for k, (ms, byts) in res.items():
        gbs = byts / (ms * 1e-3) / 1e9
        kernels[k] = {"ms_per_launch": ms, "algorithmic_bytes_per_launch": byts, "achieved_gbs": gbs,
                      "frac": gbs / HBM_PEAK_GBS}
    # measured HBM bytes per launch (profiles/<round>_pmc_hbm.json, rocprofv3
    # FETCH_SIZE / WRITE_SIZE passes over the same kernels), when committed
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_hbm.json")))
    hk = json.load(open(files[-1]))["kernels"] if files else {}
    for k in kernels:
        e = hk.get(k, {})
        # the residual leg's time includes the jagged-diagonal A x passes
        # (vector_bench times them together): so does its traffic
        kernels[k]["traffic"] = e.get("hbm_bytes_per_launch_with_row_products", e.get("hbm_bytes_per_launch"))
        kernels[k]["traffic_source"] = os.path.basename(files[-1]) if k in hk else None
    top = max(kernels, key=lambda k: kernels[k]["ms_per_launch"])
    t = kernels[top]
    return {"workload": HBM_WORKLOAD, "m": p.m, "n": p.n, "nz": p.nz, "launches_timed": reps, "kernels": kernels,
            "roofline": {"bound": "hbm", "kernel": top, "achieved": t["achieved_gbs"], "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": t["frac"], "traffic": t["traffic"]}}


def with_watchdog(seconds, fn, on_timeout):
    """fn() under a watchdog thread: after `seconds` it calls on_timeout() and
    ends the process with a non-zero code (a hang is never a success)."""
    done = threading.Event()

    def dog():
        if not done.wait(seconds):
            on_timeout()
            os._exit(WATCHDOG_EXIT)
    threading.Thread(target=dog, daemon=True).start()
    try:
        return fn()
    finally:
        done.set()


def pmc_traffic(phase):
    """HBM bytes per launch of `phase` from the newest committed PMC summary
    (profiles/<round>_pmc_traffic.json, written by tools/profile_summary.py
    from rocprofv3 FETCH_SIZE / WRITE_SIZE passes), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_traffic.json")))
    if not files:
        return None
    with open(files[-1]) as fh:
        d = json.load(fh)
    ph = d.get("phases", {}).get(phase)
    if not ph:
        return None
    return ph["hbm_bytes_per_launch"], os.path.basename(files[-1]), d.get("commit")


def pmc_mfma():
    """f64 MFMA utilisation per phase from the newest committed counter
    summary (profiles/<round>_pmc_mfma.json, tools/profile_summary.py from a
    rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_VALU_MFMA_MOPS_F64 /
    GRBM_GUI_ACTIVE pass), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, "profiles", "*_pmc_mfma.json")))
    if not files:
        return None
    with open(files[-1]) as fh:
        d = json.load(fh)
    return {"source": os.path.basename(files[-1]),
            "phases": {k: {"mfma_util": v["mfma_util"], "f64_mfma_flops_per_launch": v["f64_mfma_flops_per_launch"]}
                       for k, v in d.get("phases", {}).items()}}


def host_cpu_model():
    """The host CPU's model name (/proc/cpuinfo, as lscpu prints it)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for ln in fh:
                if ln.startswith("model name"):
                    return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def pinned(fn):
    """fn() on one host core (os.sched_setaffinity of this thread, which runs
    the oracle through ctypes), the previous mask restored after; returns
    (result, core).  The CPU legs run before the process touches the GPU."""
    old = os.sched_getaffinity(0)
    core = min(old)
    os.sched_setaffinity(0, {core})
    try:
        return fn(), core
    finally:
        os.sched_setaffinity(0, old)


def cpu_baseline(mps, iters):
    """Oracle (single-threaded C restatement of ipo) on `iters` HSD iterations
    of dfl001, pinned to one core before the GPU is initialised."""
    (_, it, loop, setup), core = pinned(lambda: oracle_run(mps, "hsd", iters))
    return {"value": it / loop, "unit": "iterations/s", "cores": 1, "kind": "port",
            "sample": f"dfl001 hsd iterations 0..{it - 1} ({it} of 117), oracle/ C restatement, "
                      f"single thread, symbolic setup {setup:.2f}s excluded, {loop:.1f}s timed",
            "pinned_core": core, "cpu_model": host_cpu_model(), "host_cpus": os.cpu_count(),
            "when": "before the GPU is initialised"}


def end_to_end(p, golden, sync):
    """SURVEY.md 8(d)'s literal definition: wall time from solver() entry to
    return (ipo_hip_solve, the same solve_impl as the `solver` symbol:
    host symbolic analysis, upload, the HSD loop, download), divided by the
    iterations printed.  One call, problem on the host at entry."""
    import ipo_amd
    sync()
    t0 = time.perf_counter()
    r = ipo_amd.solver(p, "hsd")
    el = time.perf_counter() - t0
    st = r["stats"]
    ok = r["status"] == 0 and (golden is None or abs(st["iters"] - golden) <= 1)
    return {"definition": "solver() entry to return (symbolic + upload + solve + download), host arrays in",
            "value": st["iters"] / el if ok else None, "unit": "iterations/s", "seconds": el,
            "iterations": st["iters"], "setup_s": st["t_setup_s"], "solve_s": st["t_solve_s"],
            "status": ipo_amd.STATUS_TEXT.get(r["status"], r["status"])}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5, help="timed steps: complete HSD solves to convergence (117 iterations each on dfl001)")
    ap.add_argument("--warmup", type=int, default=1, help="untimed complete solves before the timed ones")
    ap.add_argument("--problem", default="dfl001")
    ap.add_argument("--cpu-iters", type=int, default=8, help="HSD iterations of the CPU oracle sample (0 = skip)")
    ap.add_argument("--no-timing", action="store_true", help="skip the instrumented second solve (no roofline)")
    ap.add_argument("--block-angular", choices=["on", "off"], default="on",
                    help="also run BASELINE configs[4] sharded over the ranks (reported under block_angular)")
    ap.add_argument("--ba-steps", type=int, default=200, help="MAX_ITER of the block-angular solve")
    ap.add_argument("--ba-warmup", type=int, default=2, help="untimed IPM iterations before the block-angular solve")
    ap.add_argument("--ba-timeout", type=float, default=300.0, help="watchdog for the block-angular leg (s)")
    ap.add_argument("--banded", choices=["on", "off"], default="on",
                    help="also solve BASELINE configs[3] banded (factor + solve throughput, reported under banded)")
    ap.add_argument("--intpt", choices=["on", "off"], default="on",
                    help="also time BASELINE configs[1] (25fv47 by intpt, reported under intpt_25fv47)")
    ap.add_argument("--intpt-steps", type=int, default=20, help="timed complete 25fv47 intpt solves")
    ap.add_argument("--hbm", choices=["on", "off"], default="on",
                    help="also time the HBM-bound vector kernels on BASELINE configs[3] (reported under hbm_roofline)")
    args = ap.parse_args()

    d = Dist()
    import ipo_amd
    from conftest import mps_path
    path = mps_path(args.problem)
    # the CPU baselines first, each pinned to one host core, before anything
    # in this process touches the GPU (the reference CPU path
    # timed on the node's own host cores)
    cpu_hsd = cpu_intpt = None
    if d.rank == 0 and d.world == 1 and args.cpu_iters > 0:
        try:
            cpu_hsd = cpu_baseline(path, args.cpu_iters)
        except Exception as e:  # noqa: BLE001 -- the GPU number stands on its own
            cpu_hsd = {"error": repr(e)}
        if args.intpt == "on":
            try:
                cpu_intpt = intpt_cpu_baseline()
            except Exception as e:  # noqa: BLE001
                cpu_intpt = {"error": repr(e)}
    ipo_amd.require_gpu()
    if d.world > 1:
        ipo_amd.set_device(d.local)       # one process per GPU
    sync = ipo_amd.device_synchronize

    p = ipo_amd.load_mps(path)
    ctx = ipo_amd.Context(p)                       # upload + symbolic (not timed)
    golden = GOLDEN_ITERS.get(args.problem)
    for _ in range(args.warmup):
        ctx.run("hsd")
    # the timed region: K complete solves with no instrumentation

    def solves():
        return [ctx.run("hsd") for _ in range(args.steps)]
    runs, elapsed = timed_replicas(d, solves, sync)
    status, st, _ = runs[-1]
    iters = sum(r[1]["iters"] for r in runs)
    converged = all(r[0] == 0 and (golden is None or abs(r[1]["iters"] - golden) <= 1) for r in runs)
    converged = d.min(1.0 if converged else 0.0) > 0.5
    total_iters = d.sum(iters)
    value = total_iters / elapsed if converged else None
    # one more solve with per-phase HIP events on the solver's stream
    # (the events cost ~10 % of wall time, so they stay out of `value`)
    st_t, elapsed_t = st, elapsed / max(args.steps, 1)
    if not args.no_timing:
        (_, st_t, _), elapsed_t = timed_replicas(d, lambda: ctx.run("hsd", timing=True), sync)

    # dominant kernel: the phase with the most device time in the timed
    # region (HIP events on the solver's stream); algorithmic work per
    # occurrence from the symbolic plan (DESIGN.md "Kernels")
    roof, phases = None, {}
    if not args.no_timing and sum(st_t["phase_ms"]) > 0:
        for i, name in enumerate(ipo_amd.PHASES):
            ms, nl, cnt = st_t["phase_ms"][i], st_t["phase_launches"][i], st_t["phase_count"][i]
            if nl == 0 or ms <= 0:
                continue
            flops, byts = st_t["phase_flops"][i] * cnt, st_t["phase_bytes"][i] * cnt
            secs = ms * 1e-3
            phases[name] = {"kernels": PHASE_KERNELS[name], "ms_total": ms, "launches": nl,
                            "avg_launch_us": 1e3 * ms / nl, "share_of_timed_region": secs / max(elapsed_t, 1e-12),
                            "gflop_per_s": flops / secs / 1e9, "gbyte_per_s": byts / secs / 1e9,
                            "flops_per_occurrence": st_t["phase_flops"][i], "bytes_per_occurrence": st_t["phase_bytes"][i],
                            "occurrences": cnt}
        # the dominant kernel: the phase with the most device time.  Its work
        # is SURVEY.md 8(d)'s unit: the phase's share of the reference's narth
        # (ldlt.c:1243-1248; the dense tail = its columns' sum c_j^2 + 3 c_j +
        # 1), once per factorisation (a dense-tail repair's relaunches add
        # launches and time, not work); what the kernels execute (explicit
        # zeros of the widened tail, padding) is reported beside it
        top = max(phases, key=lambda k: phases[k]["ms_total"])
        ph = phases[top]
        i = ipo_amd.PHASES.index(top)
        flops_l = st_t["phase_flops"][i] * st_t["phase_count"][i] / ph["launches"]
        bytes_l = st_t["phase_bytes"][i] * st_t["phase_count"][i] / ph["launches"]
        t_l = ph["avg_launch_us"] * 1e-6
        if flops_l / (FP64_PEAK_TFLOPS * 1e12) >= bytes_l / (HBM_PEAK_GBS * 1e9):
            ach = flops_l / t_l / 1e12
            roof = {"bound": "mfma", "achieved": ach, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                    "frac": ach / FP64_PEAK_TFLOPS, "traffic": None}
        else:
            ach = bytes_l / t_l / 1e9
            roof = {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": ach / HBM_PEAK_GBS, "traffic": None}
        tr = pmc_traffic(top)
        if tr is not None:
            roof["traffic"], roof["traffic_source"], roof["traffic_commit"] = tr
            roof["traffic_note"] = "from the committed counter profile named, taken at traffic_commit, not this run"
        mf = pmc_mfma()
        if mf is not None and top in mf["phases"]:
            roof["mfma_util"] = mf["phases"][top]["mfma_util"]
            roof["mfma_source"] = mf["source"]
        roof.update({"phase": top, "kernels": ph["kernels"], "avg_launch_us": ph["avg_launch_us"],
                     "launches": ph["launches"], "occurrences": st_t["phase_count"][i],
                     "algorithmic_flops_per_occurrence": st_t["phase_flops"][i],
                     "algorithmic_flops_per_launch": flops_l,
                     "algorithmic_bytes_per_launch": bytes_l, "share_of_timed_region": ph["share_of_timed_region"],
                     "work_unit": "SURVEY.md 8(d): the phase's share of narth (ldlt.c:1243-1248) per factorisation",
                     "tail_repairs": st_t["tail_repairs"], "tail_dep_rounds": st_t["tail_dep_rounds"]})
        # executed / algorithmic per phase: f64 MFMA flops and HBM bytes from the
        # committed counter passes (profiles/<round>_pmc_{mfma,traffic}.json)
        # over the phase's algorithmic flops and bytes per launch
        for name, phd in phases.items():
            j = ipo_amd.PHASES.index(name)
            fl = st_t["phase_flops"][j] * st_t["phase_count"][j] / phd["launches"]
            by = st_t["phase_bytes"][j] * st_t["phase_count"][j] / phd["launches"]
            phd["algorithmic_flops_per_launch"], phd["algorithmic_bytes_per_launch"] = fl, by
            if mf is not None and name in mf["phases"] and fl > 0:
                phd["executed_over_algorithmic_mfma"] = mf["phases"][name]["f64_mfma_flops_per_launch"] / fl
            trn = pmc_traffic(name)
            if trn is not None and by > 0:
                phd["traffic_over_algorithmic_bytes"] = trn[0] / by
        if "executed_over_algorithmic_mfma" in ph:
            roof["executed_over_algorithmic_mfma"] = ph["executed_over_algorithmic_mfma"]
        if "traffic_over_algorithmic_bytes" in ph:
            roof["traffic_over_algorithmic_bytes"] = ph["traffic_over_algorithmic_bytes"]
        # the factor phases' algorithmic flops sum to narth (one factorisation)
        fac = sum(st_t["phase_flops"][ipo_amd.PHASES.index(k)] for k in ("gather", "diag", "trsm", "tail_syrk", "tail"))
        roof["factor_phases_sum_over_narth"] = fac / st_t["narth"] if st_t["narth"] else None

    out = {
        "metric": METRIC, "value": value, "unit": "iterations/s", "n_gpus": d.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / max(args.steps, 1), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": f"netlib {args.problem}.mps (reference problems/netlib, tests/golden copy)",
        "metric_condition_met": converged,
        "config": {"workload": f"{args.problem} hsd (BASELINE configs[2]), one step = one complete solve to mu < 1e-12",
                   "method": "hsd", "m": p.m, "n": p.n,
                   "nz": p.nz, "parallelism": f"replicas{d.world}", "status": ipo_amd.STATUS_TEXT.get(status, status),
                   "iterations_per_solve": [r[1]["iters"] for r in runs], "iterations_timed": iters,
                   "ms_per_iteration": 1e3 * elapsed / max(iters, 1),
                   "golden_iterations": golden,
                   "final_mu": st["final_mu"], "final_pobj": st["final_pobj"], "final_dobj": st["final_dobj"],
                   "setup_s": ctx.setup_seconds, "lnz": st["lnz"], "nsup": st["nsup"], "levels": st["nlevels"],
                   "factor_ms_total": st_t["factor_ms"], "solve_ms_total": st_t["solve_ms"],
                   "refine_passes": st["refine_passes"],
                   "phase_timing": "second identical solve with HIP events" if not args.no_timing else None},
        "roofline": roof,
        # the whole IPM iteration against SURVEY.md 8(d)'s algorithmic work
        # (narth + sweeps + SpMVs + vectors), over the timed region
        "iteration_roofline": (dict(roofline_of(*survey_work(st, p.m, p.n, p.nz), elapsed / max(iters, 1)),
                                    per="IPM iteration (SURVEY.md 8(d) algorithmic work), timed region")
                               if iters else None),
        "phases": phases,
        "mfma_counters": pmc_mfma(),
        "cpu_baseline": None,
    }
    if cpu_hsd is not None:
        out["cpu_baseline"] = cpu_hsd
        if value is not None and "value" in cpu_hsd:
            out["config"]["speedup_vs_cpu_baseline"] = value / cpu_hsd["value"]
    ctx.close()
    if d.rank == 0:
        try:
            out["end_to_end"] = end_to_end(p, golden, sync)
        except Exception as e:  # noqa: BLE001 -- the headline number stands on its own
            out["end_to_end"] = {"error": repr(e)}
    if args.intpt == "on" and d.world == 1:
        try:
            out["intpt_25fv47"] = intpt_leg(args, sync, cpu_intpt)
        except Exception as e:  # noqa: BLE001 -- the headline number stands on its own
            out["intpt_25fv47"] = {"workload": INTPT_WORKLOAD, "error": repr(e)}
    if args.banded == "on" and d.world == 1:
        try:
            out["banded"] = banded_leg(args)
        except Exception as e:  # noqa: BLE001 -- the headline number stands on its own
            out["banded"] = {"workload": BANDED_WORKLOAD, "error": repr(e)}
    if args.hbm == "on" and d.rank == 0:
        try:
            out["hbm_roofline"] = hbm_roofline_leg(20)
        except Exception as e:  # noqa: BLE001 -- the headline number stands on its own
            out["hbm_roofline"] = {"workload": HBM_WORKLOAD, "error": repr(e)}
    if args.block_angular == "on":
        def on_timeout():
            if d.rank == 0:
                out["block_angular"] = {"workload": BA_WORKLOAD, "error": f"timeout after {args.ba_timeout:.0f} s"}
                print(json.dumps(out), flush=True)

        def leg():
            try:
                return block_angular_leg(d, args, sync)
            except Exception as e:  # noqa: BLE001 -- the headline number stands on its own
                return {"workload": BA_WORKLOAD, "error": repr(e)}
        out["block_angular"] = with_watchdog(args.ba_timeout, leg, on_timeout)
    if d.rank == 0:
        print(json.dumps(out), flush=True)
    d.close()


if __name__ == "__main__":
    main()
