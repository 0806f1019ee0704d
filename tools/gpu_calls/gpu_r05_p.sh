#!/bin/bash
# round-5 GPU call p: packed small-leaf sweeps -- bitwise test, the GPU
# suite, the bench legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_panel.py -k "small_leaves" > gpurun_out/p_leaf.log 2>&1 || { echo leaf test failed; tail -30 gpurun_out/p_leaf.log; exit 1; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/p_suite.log 2>&1 || { echo suite failed; tail -30 gpurun_out/p_suite.log; exit 1; }
tail -2 gpurun_out/p_suite.log
timeout -k 10 400 python3 bench.py > gpurun_out/p_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/p_bench.log; exit 1; }
tail -1 gpurun_out/p_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value']); print({k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d}); print(d.get('end_to_end',{}).get('value'))"
