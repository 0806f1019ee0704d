#!/bin/bash
# round-3 GPU call S: GPU tests, then the round profile (bench default, kernel stats, PMC traffic / MFMA passes)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh 400 r03s_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
tools/gpu_step.sh 200 r03s_redo.log python3 tools/redo_stats.py linear-programming-vanderbei_amd 1 || exit 1
tools/profile_round.sh r03 || exit 1
