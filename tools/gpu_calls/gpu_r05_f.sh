#!/bin/bash
# round-5 GPU call f: one solver wave per right-hand side (tail + sparse sweeps), ticketed lead, sparse DEP,
# balanced pre-update; microbenchmark, bench, bitwise tests, GPU suite
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_step.sh 60 ub_f.log tools/ubench_tail 4441 5 || exit 1
bash tools/gpu_step.sh 60 ub_st_f.log tools/ubench_tail_st 4441 3 35 || exit 1
bash tools/gpu_step.sh 300 bench_f.log python3 bench.py --cpu-iters 0 --banded off --block-angular off --hbm off --intpt off || exit 1
bash tools/gpu_step.sh 400 f_tests.log python -u -m pytest tests/test_gpu_panel.py -x -v -s --timeout 200 --timeout-method thread -k "dependent_pivots or chain or sparse or sync_free or visit" || exit 1
bash tools/gpu_step.sh 600 gputests_f.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
