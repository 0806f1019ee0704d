#!/bin/bash
# round-3 GPU call AE: visit size A/B on configs[3] after the load fix (untimed iterations)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
for v in 32 64 128; do
IPO_HIP_VISIT_SLOTS=$v $S 200 r03ae_v$v.log python3 tools/banded_probe.py 5 0 || exit 1
done
