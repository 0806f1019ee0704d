#!/bin/bash
# Round profile on the GPU box (developer tool):
#   1. bench.py, default flags                           -> gpurun_out/<tag>_bench.log
#   2. rocprofv3 --kernel-trace --stats, dfl001 solves   -> gpurun_out/<tag>_trace/
#   3. PMC passes, one counter group each (rocprofv3 does not split passes):
#      FETCH_SIZE, WRITE_SIZE, and the f64 MFMA counters
# Every step must exit 0 (no tolerance for a non-zero profiler exit).
#   part (2nd argument): 1 = steps 1-3 and the hbm probes, 2 = the synthetic
#   legs alone (each part fits one gpurun call), all = both
tag=${1:-r04}
part=${2:-all}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
mkdir -p gpurun_out/prof_${tag}
# on a failed step: say which, drop the (large) profiler databases, stop
fail() { echo "FAILED: $1" | tee -a gpurun_out/prof_steps.txt; rm -rf gpurun_out/${tag}_trace gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write gpurun_out/${tag}_pmc_mfma gpurun_out/${tag}_pmc_hfetch gpurun_out/${tag}_pmc_hwrite gpurun_out/${tag}_banded_trace gpurun_out/${tag}_banded_pmc_* gpurun_out/${tag}_blockang_trace gpurun_out/${tag}_blockang_pmc_*; exit 1; }
if [ "$part" != 2 ]; then
B="python3 bench.py --steps 2 --warmup 0 --cpu-iters 0 --block-angular off --hbm off --banded off --intpt off"
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1 || fail bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run -- $B > gpurun_out/${tag}_trace.log 2>&1 || fail trace
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_pmc_fetch -o run -- $B --no-timing --steps 1 > gpurun_out/${tag}_pmc_fetch.log 2>&1 || fail pmc_fetch
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_pmc_write -o run -- $B --no-timing --steps 1 > gpurun_out/${tag}_pmc_write.log 2>&1 || fail pmc_write
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${tag}_pmc_mfma -o run -- $B --no-timing --steps 1 > gpurun_out/${tag}_pmc_mfma.log 2>&1 || fail pmc_mfma
# HBM traffic of the hbm_roofline leg's vector kernels (configs[3] uniform LP)
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_pmc_hfetch -o run -- python3 tools/hbm_probe.py 5 > gpurun_out/${tag}_pmc_hfetch.log 2>&1 || fail pmc_hfetch
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_pmc_hwrite -o run -- python3 tools/hbm_probe.py 5 > gpurun_out/${tag}_pmc_hwrite.log 2>&1 || fail pmc_hwrite
python3 tools/profile_summary.py ${tag} gpurun_out gpurun_out/prof_${tag} || fail summary
rm -rf gpurun_out/${tag}_trace gpurun_out/${tag}_pmc_fetch gpurun_out/${tag}_pmc_write gpurun_out/${tag}_pmc_mfma \
       gpurun_out/${tag}_pmc_hfetch gpurun_out/${tag}_pmc_hwrite
fi
[ "$part" = 1 ] && { echo profile_round $tag part 1 done; exit 0; }
# the synthetic legs: BASELINE configs[3] banded and configs[4] block-angular
# probes (5 HSD iterations each): kernel stats, FETCH / WRITE, f64 MFMA
export PROBE_ITERS=5
for leg in banded blockang; do
  P="python3 tools/${leg}_probe.py $PROBE_ITERS 0"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_${leg}_trace -o run -- $P > gpurun_out/${tag}_${leg}_trace.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_${leg}_pmc_fetch -o run -- $P > gpurun_out/${tag}_${leg}_pmc_fetch.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_${leg}_pmc_write -o run -- $P > gpurun_out/${tag}_${leg}_pmc_write.log 2>&1 || exit 1
  timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/${tag}_${leg}_pmc_mfma -o run -- $P > gpurun_out/${tag}_${leg}_pmc_mfma.log 2>&1 || exit 1
done
# the databases exceed what gpurun copies back: summarise here, keep the summaries
LEGS_ONLY=1 python3 tools/profile_summary.py ${tag} gpurun_out gpurun_out/prof_${tag} || exit 1
rm -rf gpurun_out/${tag}_banded_* gpurun_out/${tag}_blockang_*
echo profile_round $tag done
