#!/bin/bash
# round-5 GPU call d: capacity-aware visit schedule (microbenchmark on/off), eps-cap status probe, GPU suite, bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_step.sh 60 ub_sched1.log tools/ubench_tail 4441 5 || exit 1
IPO_HIP_VISIT_SCHED=0 bash tools/gpu_step.sh 60 ub_sched0.log tools/ubench_tail 4441 5 || exit 1
bash tools/gpu_step.sh 300 sched_tests.log python -u -m pytest tests/test_gpu_panel.py -x -v -s --timeout 200 --timeout-method thread -k "visit_schedule" || exit 1
bash tools/gpu_step.sh 300 bench_d.log python3 bench.py --cpu-iters 0 --banded off --block-angular off --hbm off --intpt off || exit 1
bash tools/gpu_step.sh 600 gputests_d.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread || exit 1
bash tools/gpu_step.sh 300 status_loss.log python3 tools/status_loss_probe.py gpurun_out/status_loss.json || exit 1
