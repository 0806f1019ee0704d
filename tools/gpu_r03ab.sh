#!/bin/bash
# round-3 GPU call AB: final round profile (GPU tests, bench default, kernel stats, PMC traffic / MFMA / hbm-leg passes)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh 400 r03ab_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
tools/profile_round.sh r03 || exit 1
