#!/bin/bash
# round-5 GPU call h: lead forward sweep K = 2 vs 3 (bench, A/B twice), bitwise lead test at K = 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="python3 bench.py --cpu-iters 0 --banded off --block-angular off --hbm off --intpt off"
for r in 1 2; do
IPO_HIP_LEAD_K=2 bash tools/gpu_step.sh 300 bench_h_k2_$r.log $B || exit 1
IPO_HIP_LEAD_K=3 bash tools/gpu_step.sh 300 bench_h_k3_$r.log $B || exit 1
done
IPO_HIP_LEAD_K=3 bash tools/gpu_step.sh 300 h_tests.log python -u -m pytest tests/test_gpu_panel.py -x -v -s --timeout 200 --timeout-method thread -k "chain_lead" || exit 1
