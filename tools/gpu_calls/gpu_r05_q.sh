#!/bin/bash
# round-5 GPU call q: wide panel levels split into k_diag + k_trsm -- bitwise
# test, then the bench legs with the split off / on
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_panel.py -k "split_panel" > gpurun_out/q_split.log 2>&1 || { echo split test failed; tail -30 gpurun_out/q_split.log; exit 1; }
for x in 0 768; do
IPO_HIP_PANEL_SPLIT=$x timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 > gpurun_out/q_bench_$x.log 2>&1 || { echo bench failed; tail -20 gpurun_out/q_bench_$x.log; exit 1; }
tail -1 gpurun_out/q_bench_$x.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('split=$x value', d['value']); print({k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d})"
done
