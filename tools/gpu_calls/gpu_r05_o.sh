#!/bin/bash
# round-5 GPU call o: XCD-grouped k_update chunks, A/B over the bench legs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for x in 0 1024 256; do
IPO_HIP_UPDATE_XCD=$x timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 > gpurun_out/o_bench_x$x.log 2>&1 || { echo bench failed; tail -20 gpurun_out/o_bench_x$x.log; exit 1; }
tail -1 gpurun_out/o_bench_x$x.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('x=$x value', d['value'], d.get('final_mu', d.get('config',{}).get('final_mu'))); print({k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d})"
done
