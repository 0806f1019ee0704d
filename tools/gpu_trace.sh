#!/bin/bash
# One dfl001 solve under rocprofv3 --kernel-trace, converted to CSV and broken
# down per iteration region (developer tool).  usage: gpu_trace.sh <tag> [env...]
tag=${1:-tr}; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/$tag -o run -- python3 bench.py --steps 1 --warmup 0 --no-timing --cpu-iters 0 --block-angular off > gpurun_out/$tag.log 2>&1
rc=$?; echo "trace rc=$rc"   # rocprofv3 may fault in its own finalisation after writing the DB; the DB is still complete
db=$(find gpurun_out/$tag -name "*.db" | head -1)
python3 tools/db2csv.py "$db" gpurun_out/$tag.csv && rm -rf gpurun_out/$tag && python3 tools/trace_breakdown.py gpurun_out/$tag.csv > gpurun_out/$tag.txt
grep -o '"value": [0-9.]*' gpurun_out/$tag.log
head -40 gpurun_out/$tag.txt
