#!/bin/bash
# round-3 GPU call N: one hand-off per level in the sync-free sweeps -- banded probe, dfl001 bench, tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 200 r03o_bp.log python3 tools/banded_probe.py 3 1 || exit 1
$S 300 r03o_bench.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
$S 500 r03o_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
