#!/bin/bash
# round-3 GPU call R: unconditional slot loads -- stamps, banded probe, dfl001 bench, tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
IPO_HIP_GATHER_STAMPS=2000 $S 200 gsr2000.log python3 tools/banded_probe.py 1 0 || exit 1
$S 200 r03r_bp.log python3 tools/banded_probe.py 3 1 || exit 1
$S 300 r03r_bench.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
$S 500 r03r_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
