#!/bin/bash
# round-5 GPU call aa: early dense-tail gather pieces and merged level sweeps
# -- bitwise tests, then the bench with each off / both on
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_panel.py -k "early_tail or merged_level" > gpurun_out/aa_test.log 2>&1 || { echo test failed; tail -30 gpurun_out/aa_test.log; exit 1; }
grep -c PASSED gpurun_out/aa_test.log
for cfg in "0 0" "1 0" "0 1" "1 1"; do
set -- $cfg
IPO_HIP_EARLY_TAIL=$1 IPO_HIP_MERGE_LEVELS=$2 timeout -k 10 400 python3 bench.py --intpt off --hbm off --cpu-iters 0 --banded off --block-angular off > gpurun_out/aa_bench_$1$2.log 2>&1 || { echo bench failed; tail -20 gpurun_out/aa_bench_$1$2.log; exit 1; }
tail -1 gpurun_out/aa_bench_$1$2.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); ph=d['phases']
print('early=$1 merge=$2 value', round(d['value'],1), {k:(round(v['ms_total'],1), v['launches']) for k,v in ph.items()})"
done
