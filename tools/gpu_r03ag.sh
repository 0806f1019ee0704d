#!/bin/bash
# round-3 GPU call AG: final GPU test suite + smoke on the committed tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh 500 r03ag_tests.log python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
tools/gpu_step.sh 200 r03ag_smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
