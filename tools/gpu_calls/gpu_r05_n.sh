#!/bin/bash
# round-5 GPU call n: segmented dots on the synthetic configs -- their tests,
# then the bench (banded / block-angular legs)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_synth.py tests/test_gpu_shard.py tests/test_gpu_deep.py -m gpu > gpurun_out/n_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/n_tests.log; exit 1; }
tail -3 gpurun_out/n_tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/n_bench.log 2>&1 || { echo bench failed; tail -20 gpurun_out/n_bench.log; exit 1; }
tail -1 gpurun_out/n_bench.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read())
print('value', d['value']); print({k: (d[k].get('value'), d[k].get('iterations')) for k in ('banded','block_angular') if k in d})"
