#!/bin/bash
# round-3 GPU call AC: graft smoke + the ipo_hip binary on a netlib problem
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tools/gpu_step.sh 200 r03ac_smoke.log python3 -c "import __graft_entry__ as g; g.smoke()" || exit 1
cd gpurun_out && zcat ../tests/golden/netlib/afiro.mps.gz > afiro.mps && timeout -k 10 60 ../linear-programming-vanderbei_amd/bin/ipo_hip afiro.mps hsd > r03ac_ipo.log 2>&1; echo "ipo rc=$?"; tail -5 r03ac_ipo.log; rm -f afiro.mps
