#!/bin/bash
# round-3 GPU call AD: gather chunk floor A/B on dfl001 after the unconditional-load fix
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
for c in 32 64 128 256; do
IPO_HIP_MIN_CHUNK=$c $S 300 r03ad_c$c.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
done
