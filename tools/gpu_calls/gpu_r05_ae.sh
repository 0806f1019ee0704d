#!/bin/bash
# round-5 GPU call ae (also ag): ordered dots over the non-zero products only, finish+pack folded -- the
# bitwise dot test, the GPU suite, the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dot.py > gpurun_out/ae_dot.log 2>&1 || { echo dot test failed; tail -30 gpurun_out/ae_dot.log; exit 1; }
tail -1 gpurun_out/ae_dot.log
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ae_suite.log 2>&1 || { echo suite failed; tail -30 gpurun_out/ae_suite.log; exit 1; }
tail -1 gpurun_out/ae_suite.log
timeout -k 10 400 python3 bench.py > gpurun_out/ae_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/ae_bench.log; exit 1; }
tail -1 gpurun_out/ae_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('value', round(d['value'],1), d['config'].get('final_mu'), {k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular','intpt_25fv47','end_to_end') if k in d})"
