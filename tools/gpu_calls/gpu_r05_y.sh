#!/bin/bash
# round-5 GPU call y: one dfl001 iteration's factorisation, launch by launch
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/y_trace -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-iters 0 --block-angular off --banded off --intpt off --hbm off --no-timing > gpurun_out/y_trace.log 2>&1 || { echo trace failed; tail -5 gpurun_out/y_trace.log; exit 1; }
db=$(find gpurun_out/y_trace -name '*.db' | head -1)
python3 tools/db2csv.py "$db" gpurun_out/y_kernels.csv && rm -rf gpurun_out/y_trace
python3 tools/trace_timeline.py gpurun_out/y_kernels.csv 60 400 > gpurun_out/y_timeline.txt
python3 tools/trace_timeline.py gpurun_out/y_kernels.csv 100 400 > gpurun_out/y_timeline100.txt
gzip -f gpurun_out/y_kernels.csv
wc -l gpurun_out/y_timeline.txt
