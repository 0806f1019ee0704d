#!/bin/bash
# round-5 GPU call u: dense-tail factor time by visit chunk K (ubench_tail)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for k in 6 4 5 7 8 6; do
IPO_HIP_VISIT_BLOCKS=$k timeout -k 10 60 tools/ubench_tail 4441 5 > gpurun_out/u_k$k.log 2>&1 || { echo ubench failed; tail -5 gpurun_out/u_k$k.log; exit 1; }
echo "K=$k $(grep 'per factor' gpurun_out/u_k$k.log)"
done
