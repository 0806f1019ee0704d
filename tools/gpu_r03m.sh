#!/bin/bash
# round-3 GPU call M: deep-schedule tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 400 r03n_deep.log python -u -m pytest tests/test_gpu_deep.py -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
