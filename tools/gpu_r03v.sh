#!/bin/bash
# round-3 GPU call V: paired visits + balanced dense-tail visit schedule -- microbenchmark A/B (bitwise checksums), tests, benches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
IPO_HIP_TAIL_BALANCE=0 $S 120 ubv_alap.log tools/ubench_tail 4441 5 || exit 1
$S 120 ubv_bal.log tools/ubench_tail 4441 5 || exit 1
IPO_HIP_TAIL_BALANCE=0 $S 120 ubv_alap1k.log tools/ubench_tail 1024 3 || exit 1
$S 120 ubv_bal1k.log tools/ubench_tail 1024 3 || exit 1
$S 300 r03v_bench.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
$S 500 r03v_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
