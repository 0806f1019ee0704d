#!/bin/bash
# round-3 GPU call Y: dfl001 with the deep-tree schedule forced (visits + quadrant gathers + forward pre-pass)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
IPO_HIP_VISITS=1 $S 300 r03y_visits.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
IPO_HIP_GATHER_FLAT=2 $S 300 r03y_flat2.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
$S 300 r03y_base.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
$S 200 r03y_hbm.log python3 tools/hbm_probe.py 5 || exit 1
