"""Turn the rocprofv3 databases of tools/profile_round.sh into the files
committed under profiles/ (developer tool).

  profiles/<tag>_kernel_stats.csv   top_kernels of the --kernel-trace --stats run
                                    (name, calls, total_us, avg_us, percent)
  profiles/<tag>_pmc_traffic.json   HBM bytes per launch from the FETCH_SIZE /
                                    WRITE_SIZE passes, per kernel and per phase
  profiles/<tag>_bench.json         the bench.py JSON line of the same run

FETCH_SIZE on gfx950 counts half of the bytes of wide streaming reads
(MI355X_MICROARCH.md, HBM section): it is doubled here; WRITE_SIZE is taken
as reported.  Both are KB in rocprofv3.
  profiles/<tag>_tail_steps.json   k_tail_pr durations in dispatch order (the
                                    first 700: ten factorisations' look-ahead steps)
  profiles/<tag>_{banded,blockang}_kernel_stats.csv, _profile.json
                                    the synthetic legs' probes: kernel stats, HBM
                                    bytes and f64 MFMA flops per IPM iteration
usage: python tools/profile_summary.py r01 [gpurun_out] [profiles dir]"""
import csv
import json
import os
import re
import sqlite3
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from bench import PHASE_KERNELS  # noqa: E402

tag = sys.argv[1]
src = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "gpurun_out")
dst = sys.argv[3] if len(sys.argv) > 3 else os.path.join(REPO, "profiles")
os.makedirs(dst, exist_ok=True)


LEGS_ONLY = os.environ.get("LEGS_ONLY") == "1"     # tools/profile_round.sh part 2: the synthetic legs alone
# the commit the profiled tree was taken at (the GPU box has no .git: the
# caller passes it, tools/gpu_recipes.sh profile); recorded in every summary
COMMIT = os.environ.get("PROFILE_COMMIT")


def short(name):
    return name.replace("ipo::(anonymous namespace)::", "").replace("ipo::", "").split("(")[0]


def per_kernel(db, counter):
    c = sqlite3.connect(db)
    acc = {}
    for name, val in c.execute("select kernel_name, value from counters_collection where counter_name = ?",
                               (counter,)):
        k = short(name)
        s, n = acc.get(k, (0.0, 0))
        acc[k] = (s + val, n + 1)
    return acc


def base(k):
    """kernel name without 'void ' and template arguments (the PHASE_KERNELS names)"""
    return re.sub(r"<.*>", "", k.replace("void ", "")).strip()


def dfl001_part():
    c = sqlite3.connect(os.path.join(src, f"{tag}_trace", "run_results.db"))
    rows = list(c.execute("select name, total_calls, total_duration, average, percentage from top_kernels "
                          "order by total_duration desc"))
    with open(os.path.join(dst, f"{tag}_kernel_stats.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for n, calls, tot, avg, pct in rows:
            w.writerow([short(n), calls, f"{tot:.1f}", f"{avg:.2f}", f"{pct:.2f}"])


    steps = [round((e - b) / 1000.0, 1) for b, e in
             c.execute("select start, end from kernels where name like '%k_tail_pr%' order by start limit 700")]
    runs = [round((e - b) / 1000.0, 1) for b, e in
            c.execute("select start, end from kernels where name like '%k_tail_run%' order by start limit 200")]
    with open(os.path.join(dst, f"{tag}_tail_steps.json"), "w") as fh:
        json.dump({"source": "rocprofv3 --kernel-trace, bench.py --steps 2 (dfl001 hsd)", "unit": "us", "commit": COMMIT,
                   "k_tail_pr": steps, "k_tail_run": runs}, fh)


    fetch = per_kernel(os.path.join(src, f"{tag}_pmc_fetch", "run_results.db"), "FETCH_SIZE")
    write = per_kernel(os.path.join(src, f"{tag}_pmc_write", "run_results.db"), "WRITE_SIZE")
    kern = {}
    for k in sorted(set(fetch) | set(write)):
        fs, fn = fetch.get(k, (0.0, 0))
        ws, wn = write.get(k, (0.0, 0))
        n = max(fn, wn, 1)
        kern[k] = {"launches": n, "fetch_bytes_per_launch": 2 * 1024 * fs / max(fn, 1),
                   "write_bytes_per_launch": 1024 * ws / max(wn, 1)}
        kern[k]["hbm_bytes_per_launch"] = kern[k]["fetch_bytes_per_launch"] + kern[k]["write_bytes_per_launch"]
    phases = {}
    for ph, names in PHASE_KERNELS.items():
        want = set(re.split(r"[|+]", names))
        ks = [k for k in kern if base(k) in want]
        tot = sum(kern[k]["hbm_bytes_per_launch"] * kern[k]["launches"] for k in ks)
        nl = sum(kern[k]["launches"] for k in ks)
        if nl:
            phases[ph] = {"kernels": ks, "launches": nl, "hbm_bytes_per_launch": tot / nl}
    with open(os.path.join(dst, f"{tag}_pmc_traffic.json"), "w") as fh:
        json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, bench.py --steps 1 --warmup 0 --no-timing "
                             "(dfl001 hsd, first 10 iterations); FETCH_SIZE doubled (gfx950)",
                   "commit": COMMIT, "phases": phases, "kernels": kern}, fh, indent=1)
    # f64 MFMA utilisation per kernel / phase: SQ_VALU_MFMA_BUSY_CYCLES (MFMA-busy
    # cycles summed over the SIMDs: 64 per v_mfma_f64_16x16x4f64, calibrated on
    # k_tail_pr whose instruction count is known) over the kernel's active
    # cycles x SIMDs (1,024 on MI355X: 256 CUs x 4), the active cycles being
    # GRBM_GUI_ACTIVE / 8 -- the counter sums the 8 XCDs (GRBM_GUI_ACTIVE / 8 at
    # ~2.4-2.8 GHz is the kernel's trace duration); f64 MFMA flops from
    # SQ_INSTS_VALU_MFMA_MOPS_F64 (units of 512 flops: 431 MFLOP per k_tail_pr
    # launch = the algorithmic count) over the kernel's trace duration (us)
    mdb = os.path.join(src, f"{tag}_pmc_mfma", "run_results.db")
    if os.path.exists(mdb):
        SIMDS, XCDS = 1024, 8
        busy = per_kernel(mdb, "SQ_VALU_MFMA_BUSY_CYCLES")
        mops = per_kernel(mdb, "SQ_INSTS_VALU_MFMA_MOPS_F64")
        gui = per_kernel(mdb, "GRBM_GUI_ACTIVE")
        sqb = per_kernel(mdb, "SQ_BUSY_CYCLES")
        dur = {short(n): avg for n, _, _, avg, _ in rows}     # us per launch, kernel-trace run
        mk = {}
        for k in busy:
            b, n = busy[k]
            g = gui.get(k, (0.0, 1))[0]
            mo = mops.get(k, (0.0, 1))[0]
            mk[k] = {"launches": n, "mfma_busy_cycles": b / n, "gui_active_cycles": g / n,
                     "mfma_util": b / (g / XCDS * SIMDS) if g else None, "f64_mfma_flops_per_launch": 512.0 * mo / n,
                     "sq_busy_cycles": sqb.get(k, (0.0, 1))[0] / n}
            if k in dur and dur[k]:
                mk[k]["f64_mfma_tflops"] = mk[k]["f64_mfma_flops_per_launch"] / (dur[k] * 1e-6) / 1e12
        mph = {}
        for ph, names in PHASE_KERNELS.items():
            want = set(re.split(r"[|+]", names))
            ks = [k for k in mk if base(k) in want]
            b = sum(mk[k]["mfma_busy_cycles"] * mk[k]["launches"] for k in ks)
            g = sum(mk[k]["gui_active_cycles"] * mk[k]["launches"] for k in ks)
            f = sum(mk[k]["f64_mfma_flops_per_launch"] * mk[k]["launches"] for k in ks)
            nl = sum(mk[k]["launches"] for k in ks)
            if nl:
                mph[ph] = {"kernels": ks, "launches": nl, "mfma_util": b / (g / XCDS * SIMDS) if g else None,
                           "f64_mfma_flops_per_launch": f / nl}
        with open(os.path.join(dst, f"{tag}_pmc_mfma.json"), "w") as fh:
            json.dump({"source": "rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES "
                                 "GRBM_GUI_ACTIVE, bench.py --steps 1 --warmup 0 --no-timing (dfl001 hsd); util = "
                                 "MFMA-busy cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs); MOPS_F64 in units of 512 "
                                 "flops; tflops over the kernel-trace average duration",
                       "commit": COMMIT, "phases": mph, "kernels": mk}, fh, indent=1)
    # HBM bytes per launch of the hbm_roofline leg's kernels (tools/hbm_probe.py
    # under the same FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE doubled)
    hf = os.path.join(src, f"{tag}_pmc_hfetch", "run_results.db")
    if os.path.exists(hf):
        hfetch = per_kernel(hf, "FETCH_SIZE")
        hwrite = per_kernel(os.path.join(src, f"{tag}_pmc_hwrite", "run_results.db"), "WRITE_SIZE")
        hk = {}
        for k in sorted(set(hfetch) | set(hwrite)):
            kb = base(k)
            if kb not in ("k_hsd_residuals", "k_rows_ax_jds", "k_hsd_directions", "k_step"):
                continue
            fs, fn = hfetch.get(k, (0.0, 0))
            ws, wn = hwrite.get(k, (0.0, 0))
            hk[kb] = {"launches": max(fn, wn), "fetch_bytes_per_launch": 2 * 1024 * fs / max(fn, 1),
                      "write_bytes_per_launch": 1024 * ws / max(wn, 1)}
            hk[kb]["hbm_bytes_per_launch"] = hk[kb]["fetch_bytes_per_launch"] + hk[kb]["write_bytes_per_launch"]
        # the residual leg is A x by jagged diagonals (large x) + the residual
        # kernel: its traffic per residual launch is the sum of both
        if "k_rows_ax_jds" in hk and "k_hsd_residuals" in hk:
            r, j = hk["k_hsd_residuals"], hk["k_rows_ax_jds"]
            per = j["launches"] / max(r["launches"], 1)
            r["hbm_bytes_per_launch_with_row_products"] = r["hbm_bytes_per_launch"] + per * j["hbm_bytes_per_launch"]
        with open(os.path.join(dst, f"{tag}_pmc_hbm.json"), "w") as fh:
            json.dump({"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE, tools/hbm_probe.py 5 (bench.py's "
                                 "hbm_roofline kernels, BASELINE configs[3] uniform LP); FETCH_SIZE doubled (gfx950)",
                       "commit": COMMIT, "kernels": hk}, fh, indent=1)


if not LEGS_ONLY:
    dfl001_part()
# the synthetic legs (BASELINE configs[3] banded, configs[4] block-angular):
# kernel stats and HBM traffic / f64 MFMA per IPM iteration of a probe run
# (tools/banded_probe.py, tools/blockang_probe.py, ITERS iterations, setup
# uploads are copies, not kernels)
for leg, probe in (("banded", "tools/banded_probe.py"), ("blockang", "tools/blockang_probe.py")):
    tdb = os.path.join(src, f"{tag}_{leg}_trace", "run_results.db")
    if not os.path.exists(tdb):
        continue
    iters = int(os.environ.get("PROBE_ITERS", "5"))
    c2 = sqlite3.connect(tdb)
    krows = list(c2.execute("select name, total_calls, total_duration, average, percentage from top_kernels "
                            "order by total_duration desc"))
    with open(os.path.join(dst, f"{tag}_{leg}_kernel_stats.csv"), "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for n, calls, tot, avg, pct in krows:
            w.writerow([short(n), calls, f"{tot:.1f}", f"{avg:.2f}", f"{pct:.2f}"])
    out = {"source": f"rocprofv3 --kernel-trace --stats / --pmc passes, python3 {probe} {iters} 0; FETCH_SIZE "
                     f"doubled (gfx950); per IPM iteration = run total / {iters}",
           "iterations": iters, "kernel_ms_per_iteration": sum(r[2] for r in krows) / 1000.0 / iters, "commit": COMMIT}
    f_ = os.path.join(src, f"{tag}_{leg}_pmc_fetch", "run_results.db")
    w_ = os.path.join(src, f"{tag}_{leg}_pmc_write", "run_results.db")
    if os.path.exists(f_) and os.path.exists(w_):
        fe, wr = per_kernel(f_, "FETCH_SIZE"), per_kernel(w_, "WRITE_SIZE")
        out["hbm_bytes_per_iteration"] = (2 * 1024 * sum(v for v, _ in fe.values())
                                          + 1024 * sum(v for v, _ in wr.values())) / iters
        top = {}
        for k in sorted(set(fe) | set(wr), key=lambda k: -(fe.get(k, (0, 0))[0] * 2 + wr.get(k, (0, 0))[0]))[:12]:
            top[k] = (2 * 1024 * fe.get(k, (0.0, 0))[0] + 1024 * wr.get(k, (0.0, 0))[0]) / iters
        out["hbm_bytes_per_iteration_top_kernels"] = top
    m_ = os.path.join(src, f"{tag}_{leg}_pmc_mfma", "run_results.db")
    if os.path.exists(m_):
        SIMDS, XCDS = 1024, 8
        bu, mo, gu = (per_kernel(m_, k) for k in ("SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F64",
                                                  "GRBM_GUI_ACTIVE"))
        b = sum(v for v, _ in bu.values())
        g = sum(v for v, _ in gu.values())
        out["f64_mfma_flops_per_iteration"] = 512.0 * sum(v for v, _ in mo.values()) / iters
        out["mfma_util_over_kernel_time"] = b / (g / XCDS * SIMDS) if g else None
    with open(os.path.join(dst, f"{tag}_{leg}_profile.json"), "w") as fh:
        json.dump(out, fh, indent=1)
if not LEGS_ONLY:
    line = [ln for ln in open(os.path.join(src, f"{tag}_bench.log")) if ln.startswith("{")][-1]
    with open(os.path.join(dst, f"{tag}_bench.json"), "w") as fh:
        fh.write(line)
    print("wrote", dst)
