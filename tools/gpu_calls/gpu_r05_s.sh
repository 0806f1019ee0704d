#!/bin/bash
# round-5 GPU call s: single-column small panels eight to a wave -- bitwise
# test, then the bench legs with them off / on
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_panel.py -k "small_leaves or split_panel" > gpurun_out/s_test.log 2>&1 || { echo test failed; tail -30 gpurun_out/s_test.log; exit 1; }
grep -c PASSED gpurun_out/s_test.log
for x in 0 32768; do
IPO_HIP_SMALL_LEAVES=$x timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 > gpurun_out/s_bench_$x.log 2>&1 || { echo bench failed; tail -20 gpurun_out/s_bench_$x.log; exit 1; }
tail -1 gpurun_out/s_bench_$x.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('small=$x value', round(d['value'],1), {k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d})"
done
