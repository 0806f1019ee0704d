#!/bin/bash
# round-3 GPU call I: banded configs[3] chain probe (phases + kernel trace of 2 iterations)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 200 bp_phases.log python3 tools/banded_probe.py 3 1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/bp_tr -o run -- python3 tools/banded_probe.py 2 0 > gpurun_out/bp_tr.log 2>&1 || exit 1
db=$(find gpurun_out/bp_tr -name "*.db" | head -1)
python3 tools/db2csv.py "$db" gpurun_out/bp_tr.csv && rm -rf gpurun_out/bp_tr && python3 tools/chain_trace.py gpurun_out/bp_tr.csv > gpurun_out/bp_chain.txt
cat gpurun_out/bp_chain.txt | head -50
