#!/bin/bash
# round-3 GPU call AF: dense-tail density threshold re-measured on dfl001 after the gather load fix
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
for d in 0.6 0.8 0.9; do
IPO_HIP_TAIL_DENSITY=$d $S 300 r03af_d$d.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
done
