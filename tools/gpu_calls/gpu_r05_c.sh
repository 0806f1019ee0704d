#!/bin/bash
# round-5 GPU call c: panel window hand-off stamps (base / eager apply), status-loss probe with the eps cap, redo counts
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
zcat tests/golden/netlib/dfl001.mps.gz > /tmp/dfl001.mps || exit 1
bash tools/gpu_step.sh 60 ub_st_base.log tools/ubench_tail_st 4441 3 35 || exit 1
bash tools/gpu_step.sh 60 ub_st_e1.log tools/ubench_tail_st_e1 4441 3 35 || exit 1
bash tools/gpu_step.sh 60 ub_e1.log tools/ubench_tail_e1 4441 5 || exit 1
bash tools/gpu_step.sh 60 ub_base.log tools/ubench_tail 4441 5 || exit 1
IPO_HIP_DEBUG_REDO=1 bash tools/gpu_step.sh 60 redo.log linear-programming-vanderbei_amd/bin/ipo_hip /tmp/dfl001.mps || exit 1
bash tools/gpu_step.sh 500 status_loss.log python3 tools/status_loss_probe.py gpurun_out/status_loss.json || exit 1
