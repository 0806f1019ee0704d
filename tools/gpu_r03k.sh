#!/bin/bash
# round-3 GPU call K: banded kernel trace with visits, visit size A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/bp2_tr -o run -- python3 tools/banded_probe.py 2 0 > gpurun_out/bp2_tr.log 2>&1 || exit 1
db=$(find gpurun_out/bp2_tr -name "*.db" | head -1)
python3 tools/db2csv.py "$db" gpurun_out/bp2_tr.csv && rm -rf gpurun_out/bp2_tr && python3 tools/chain_trace.py gpurun_out/bp2_tr.csv > gpurun_out/bp2_chain.txt
head -30 gpurun_out/bp2_chain.txt
for v in 32 128 256; do
IPO_HIP_VISIT_SLOTS=$v $S 200 r03l_bp_v$v.log python3 tools/banded_probe.py 3 1 || exit 1
done
