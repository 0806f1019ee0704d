#!/bin/bash
# round-5 GPU call z: the dense tail's gather in early pieces -- bitwise
# tests, the bench with it off / on, one factorisation's timeline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_panel.py -k "early_tail" > gpurun_out/z_test.log 2>&1 || { echo test failed; tail -30 gpurun_out/z_test.log; exit 1; }
grep -c PASSED gpurun_out/z_test.log
for x in 0 1; do
IPO_HIP_EARLY_TAIL=$x timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 > gpurun_out/z_bench_$x.log 2>&1 || { echo bench failed; tail -20 gpurun_out/z_bench_$x.log; exit 1; }
tail -1 gpurun_out/z_bench_$x.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('early=$x value', round(d['value'],1), {k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d})"
done
