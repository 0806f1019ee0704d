#!/bin/bash
# GPU-call recipes (developer tool): every gpurun call of a development
# round is one of these, run from the repository root on the GPU box as
#   gpurun --timeout S -- 'bash tools/gpu_recipes.sh <recipe> [args]'
# so that a number quoted in DESIGN.md or a commit message can be traced to
# the steps that produced it (round 5's one-off call scripts, tools/gpu_calls/,
# are in the history before this file replaced them).  Each GPU step runs under its own time limit
# (tools/gpu_step.sh: a fault, abort or timeout stops the call there) and
# writes its log under gpurun_out/.  The round profile is tools/profile_round.sh.
#
# recipes:
#   ubtail [nt]      the dense-tail microbenchmark (tools/ubench_tail, built on
#                    the CPU side): per-step launches, then the persistent run
#                    (k_tail_run) against them; nt 2000 adds the host LDL' check
#   panel            tests/test_gpu_panel.py (bitwise variant tests of the factor)
#   suite            the whole GPU suite (pytest -m gpu)
#   bench [args]     bench.py (dfl001 only unless args say otherwise)
#   ab VAR v0 v1     bench.py dfl001 with VAR=v0, then VAR=v1, twice each
#   sweep            tools/gpu_sweep.py over every problem (hsd) and the intpt /
#                    hsdls sets, traces saved (offline parity checks)
#   profile TAG [p]  tools/profile_round.sh TAG [part]; pass the commit the tree
#                    was taken at as PROFILE_COMMIT=<sha> before the recipe
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
STEP="bash tools/gpu_step.sh"
B1="python3 bench.py --cpu-iters 0 --banded off --block-angular off --hbm off --intpt off"
PYT="python3 -u -m pytest -x -q --timeout 300 --timeout-method thread"

recipe=$1; shift
case "$recipe" in
ubtail)
    nt=${1:-4441}
    # the microbenchmark binary does not travel (.gpurunignore): built here
    [ -x tools/ubench_tail ] || hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off \
        -I linear-programming-vanderbei_amd/csrc tools/ubench_tail.hip -o tools/ubench_tail || exit 1
    $STEP 60 ub_step_$nt.log tools/ubench_tail $nt 5 || exit 1
    UB_RUN=1 $STEP 60 ub_run_$nt.log tools/ubench_tail $nt 5 || exit 1
    ;;
panel)
    $STEP 600 panel.log $PYT tests/test_gpu_panel.py || exit 1
    ;;
suite)
    $STEP 1100 suite.log $PYT tests -m gpu || exit 1
    ;;
bench)
    if [ $# -gt 0 ]; then $STEP 400 bench.log python3 bench.py "$@" || exit 1
    else $STEP 400 bench.log $B1 || exit 1; fi
    ;;
ab)
    var=$1; v0=$2; v1=$3
    for r in 1 2; do
        env "$var=$v0" $STEP 300 ab_${var}_${v0}_$r.log $B1 || exit 1
        env "$var=$v1" $STEP 300 ab_${var}_${v1}_$r.log $B1 || exit 1
    done
    ;;
sweep)
    # every netlib problem by HSD, the intpt / hsdls sets by their methods
    # (tools/gpu_sweep.py); traces under gpurun_out/sweep_<method>/
    ONLY=$(python3 -c "import sys; sys.path.insert(0, 'tools'); from rounding_stability import INTPT_SET; print(','.join(INTPT_SET))")
    SWEEP_SAVE=gpurun_out/sweep_hsd $STEP 600 sweep_hsd.jsonl python3 tools/gpu_sweep.py || exit 1
    for m in intpt hsdls; do
        SWEEP_METHOD=$m SWEEP_ONLY=$ONLY SWEEP_SAVE=gpurun_out/sweep_$m $STEP 400 sweep_$m.jsonl python3 tools/gpu_sweep.py || exit 1
    done
    ;;
profile)
    bash tools/profile_round.sh "$@" || exit 1
    ;;
*)
    echo "unknown recipe $recipe"; exit 2
    ;;
esac
