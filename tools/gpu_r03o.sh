#!/bin/bash
# round-3 GPU call O: banded kernel traces, flat gather vs pipelined, visit size 256
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tr() {   # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$tag -o run -- python3 tools/banded_probe.py 1 0 > gpurun_out/$tag.log 2>&1 || return 1
  db=$(find gpurun_out/$tag -name "*.db" | head -1)
  python3 tools/db2csv.py "$db" gpurun_out/$tag.csv && rm -rf gpurun_out/$tag && python3 tools/chain_trace.py gpurun_out/$tag.csv > gpurun_out/$tag.txt
}
tr bpf_flat IPO_HIP_GATHER_FLAT=1 || exit 1
tr bpf_pipe IPO_HIP_GATHER_FLAT=0 || exit 1
tr bpf_flat256 IPO_HIP_GATHER_FLAT=1 IPO_HIP_VISIT_SLOTS=256 || exit 1
head -8 gpurun_out/bpf_flat.txt gpurun_out/bpf_pipe.txt gpurun_out/bpf_flat256.txt
