#!/bin/bash
# round-5 first GPU call: tail microbenchmark (+ stamps of a middle and a late step), the GPU tests, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_step.sh 60 ub_tail.log tools/ubench_tail 4441 5 || exit 1
bash tools/gpu_step.sh 60 ub_tail_st35.log tools/ubench_tail_st 4441 3 35 || exit 1
bash tools/gpu_step.sh 60 ub_tail_st66.log tools/ubench_tail_st 4441 3 66 || exit 1
bash tools/gpu_step.sh 600 gputests.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread || exit 1
bash tools/gpu_step.sh 400 bench.log python3 bench.py || exit 1
bash tools/gpu_step.sh 500 status_loss.log python3 tools/status_loss_probe.py gpurun_out/status_loss.json || exit 1
