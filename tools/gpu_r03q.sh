#!/bin/bash
# round-3 GPU call Q: quadrant gather -- stamps, banded probe, deep tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
IPO_HIP_GATHER_STAMPS=2000 $S 200 gsq2000.log python3 tools/banded_probe.py 1 0 || exit 1
$S 200 r03q_bp.log python3 tools/banded_probe.py 3 1 || exit 1
$S 400 r03q_deep.log python -u -m pytest tests/test_gpu_deep.py -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
$S 200 r03q_redo.log python3 tools/redo_stats.py linear-programming-vanderbei_amd 1 || exit 1
