#!/bin/bash
# round-5 GPU call b: in-panel dependent pivots (tail microbenchmark, bitwise tests, bench)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_step.sh 60 ub_tail_b.log tools/ubench_tail 4441 5 || exit 1
bash tools/gpu_step.sh 400 spec_tests.log python -u -m pytest tests/test_gpu_panel.py -x -v -s --timeout 200 --timeout-method thread -k "dependent_pivots or tail_repair" || exit 1
bash tools/gpu_step.sh 300 bench_b.log python3 bench.py --cpu-iters 0 --banded off --block-angular off --hbm off --intpt off || exit 1
