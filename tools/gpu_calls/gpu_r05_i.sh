#!/bin/bash
# round-5 GPU call i: lead forward sweep stamps (lib_st built with -DIPO_LEAD_STAMPS), then the round profile part 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
zcat tests/golden/netlib/dfl001.mps.gz > /tmp/dfl001.mps || exit 1
LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/linear-programming-vanderbei_amd/lib_st bash tools/gpu_step.sh 120 lead_st.log linear-programming-vanderbei_amd/bin_st/ipo_hip /tmp/dfl001.mps || exit 1
bash tools/profile_round.sh r05 1
