#!/bin/bash
# exit-time fault under rocprofv3 (developer tool): one run, its mappings kept
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
P=${1:-dfl001}; M=${2:-plain}
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ep_$M -o run -- python3 tools/exit_probe.py $M $P 2 gpurun_out/ep_maps_$M.txt > gpurun_out/ep_$M.log 2>&1
rc=$?; echo "$M $P rc=$rc" >> gpurun_out/ep.txt
