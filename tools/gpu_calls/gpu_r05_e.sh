#!/bin/bash
# round-5 GPU call e: one solver wave per right-hand side in the tail sweeps; sparse DEP tests; bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_step.sh 300 bench_e.log python3 bench.py --cpu-iters 0 --banded off --block-angular off --hbm off --intpt off || exit 1
bash tools/gpu_step.sh 400 e_tests.log python -u -m pytest tests/test_gpu_panel.py -x -v -s --timeout 200 --timeout-method thread -k "dependent_pivots or chain or sparse" || exit 1
