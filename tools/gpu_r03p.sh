#!/bin/bash
# round-3 GPU call P: gather stamps on chain levels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
IPO_HIP_GATHER_STAMPS=2000 $S 200 gst2000.log python3 tools/banded_probe.py 1 0 || exit 1
IPO_HIP_GATHER_STAMPS=2000 IPO_HIP_VISIT_SLOTS=256 $S 200 gst2000_256.log python3 tools/banded_probe.py 1 0 || exit 1
