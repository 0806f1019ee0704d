#!/bin/bash
# round-5 GPU call k: XCD-grouped visits (microbenchmark A/B, twice)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for r in 1 2; do
IPO_HIP_VISIT_XCD=0 bash tools/gpu_step.sh 60 ub_k_x0_$r.log tools/ubench_tail 4441 5 || exit 1
IPO_HIP_VISIT_XCD=1 bash tools/gpu_step.sh 60 ub_k_x1_$r.log tools/ubench_tail 4441 5 || exit 1
done
