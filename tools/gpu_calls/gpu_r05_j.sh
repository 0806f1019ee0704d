#!/bin/bash
# round-5 GPU call j: backward dense-tail sweep by a lead workgroup (A/B against the chain), GPU suite
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
B="python3 bench.py --cpu-iters 0 --banded off --block-angular off --hbm off --intpt off"
IPO_HIP_BWD_LEAD=1 bash tools/gpu_step.sh 300 bench_j_lead.log $B || exit 1
IPO_HIP_BWD_LEAD=0 bash tools/gpu_step.sh 300 bench_j_chain.log $B || exit 1
bash tools/gpu_step.sh 900 gputests_j.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
