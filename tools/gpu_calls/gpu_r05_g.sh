#!/bin/bash
# round-5 GPU call g: pre-update A/B (HEAD vs templated fragments), stamps, setup times
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
zcat tests/golden/netlib/dfl001.mps.gz > /tmp/dfl001.mps || exit 1
for r in 1 2; do
bash tools/gpu_step.sh 60 ub_g_head$r.log tools/ubench_tail_head 4441 5 || exit 1
bash tools/gpu_step.sh 60 ub_g_new$r.log tools/ubench_tail 4441 5 || exit 1
done
bash tools/gpu_step.sh 60 ub_st_g_head.log tools/ubench_tail_st_head 4441 3 35 || exit 1
bash tools/gpu_step.sh 60 ub_st_g_new.log tools/ubench_tail_st 4441 3 35 || exit 1
IPO_HIP_SETUP_TIMES=1 bash tools/gpu_step.sh 60 setup_times.log linear-programming-vanderbei_amd/bin/ipo_hip /tmp/dfl001.mps || exit 1
