#!/bin/bash
# round-3 GPU call Z: one launch per chain level (k_level) -- A/B bitwise probe, deep tests, all tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 300 r03z_deep.log python -u -m pytest tests/test_gpu_deep.py -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
IPO_HIP_LEVEL_FUSE=0 $S 200 r03z_bp0.log python3 tools/banded_probe.py 3 1 || exit 1
$S 200 r03z_bp1.log python3 tools/banded_probe.py 3 1 || exit 1
$S 500 r03z_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
