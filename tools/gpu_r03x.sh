#!/bin/bash
# round-3 GPU call X: segmented long dots -- banded bench leg, GPU tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 600 r03x_bench.log python3 bench.py --steps 3 --warmup 1 --cpu-iters 0 --block-angular on --hbm off --banded on || exit 1
$S 500 r03x_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
