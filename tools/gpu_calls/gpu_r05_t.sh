#!/bin/bash
# round-5 GPU call t: the wide gather (k_update<4>) at 3 workgroups per CU
# (168 VGPRs, 16 spilled) against 2 (244 VGPRs) over the bench legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for x in 0 1; do
IPO_HIP_UPDATE_WIDE_OCC=$x timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 > gpurun_out/t_bench_$x.log 2>&1 || { echo bench failed; tail -20 gpurun_out/t_bench_$x.log; exit 1; }
tail -1 gpurun_out/t_bench_$x.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('wide=$x value', round(d['value'],1), {k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d}, 'gather', round(ph['gather']['ms_total'],1))"
done
