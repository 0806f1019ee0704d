#!/bin/bash
# round-5 GPU call af: the HBM leg's residual (JDS row products + residual)
# by the number of column slices of A x
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for b in 1 2 4 8; do
echo "blocks $b: $(IPO_HIP_AX_BLOCKS=$b timeout -k 10 120 python3 tools/hbm_probe.py 20)"
done
