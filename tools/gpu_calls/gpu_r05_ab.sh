#!/bin/bash
# round-5 GPU call ab: early dense-tail gather pieces at the lowest stream
# priority (the solver's stream at the highest), merged sweeps on
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for x in 0 1; do
IPO_HIP_DEBUG_PRIO=1 IPO_HIP_EARLY_TAIL=$x timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 --banded off --block-angular off > gpurun_out/ab_bench_$x.log 2>&1 || { echo bench failed; tail -20 gpurun_out/ab_bench_$x.log; exit 1; }
grep -m1 "stream priorities" gpurun_out/ab_bench_$x.log
tail -1 gpurun_out/ab_bench_$x.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('early=$x value', round(d['value'],1), {k:(round(v['ms_total'],1), v['launches']) for k,v in ph.items()})"
done
