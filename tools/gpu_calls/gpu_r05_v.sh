#!/bin/bash
# round-5 GPU call v: HSD residual with paired items -- GPU suite, then the
# bench (HBM leg)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/v_suite.log 2>&1 || { echo suite failed; tail -30 gpurun_out/v_suite.log; exit 1; }
tail -2 gpurun_out/v_suite.log
timeout -k 10 400 python3 bench.py > gpurun_out/v_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/v_bench.log; exit 1; }
tail -1 gpurun_out/v_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', round(d['value'],1), {k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d}, 'e2e', d['end_to_end']['value'])
h=d['hbm_roofline']; print(json.dumps(h)[:1500])"
