#!/bin/bash
# round-5 GPU call x: wide gathers (four partials at a time, 2 per CU) on / off
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for x in 1 0; do
IPO_HIP_GATHER_WIDE=$x timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 > gpurun_out/x_bench_$x.log 2>&1 || { echo bench failed; tail -20 gpurun_out/x_bench_$x.log; exit 1; }
tail -1 gpurun_out/x_bench_$x.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('wide=$x value', round(d['value'],1), {k: (d[k].get('value'), d[k].get('iterations'), d[k].get('final_mu')) for k in ('banded','block_angular') if k in d}, 'gather', round(ph['gather']['ms_total'],1))"
done
