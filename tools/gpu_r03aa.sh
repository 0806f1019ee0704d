#!/bin/bash
# round-3 GPU call AA: k_level with 64-slot rounds -- deep tests, probes A/B, banded bench leg
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 300 r03aa_deep.log python -u -m pytest tests/test_gpu_deep.py -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
IPO_HIP_LEVEL_FUSE=0 $S 200 r03aa_bp0.log python3 tools/banded_probe.py 3 1 || exit 1
$S 200 r03aa_bp1.log python3 tools/banded_probe.py 3 1 || exit 1
$S 600 r03aa_bench.log python3 bench.py --steps 3 --warmup 1 --cpu-iters 0 --block-angular on --hbm off --banded on || exit 1
