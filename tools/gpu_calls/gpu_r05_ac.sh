#!/bin/bash
# round-5 GPU call ac (also ad): refinement passes with both systems per launch, merged panels -- the
# GPU suite (golden traces, bitwise comparisons), then the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ac_suite.log 2>&1 || { echo suite failed; tail -30 gpurun_out/ac_suite.log; exit 1; }
tail -2 gpurun_out/ac_suite.log
timeout -k 10 400 python3 bench.py > gpurun_out/ac_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/ac_bench.log; exit 1; }
tail -1 gpurun_out/ac_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('value', round(d['value'],1), d['config'].get('final_mu'), {k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular','intpt_25fv47','end_to_end') if k in d})
print({k:(round(v['ms_total'],1), v['launches']) for k,v in ph.items()})"
