#!/bin/bash
# round-5 GPU call l: XCD-grouped visits in the library -- bitwise tests,
# the whole GPU suite, the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_panel.py -k "visit_schedule" > gpurun_out/l_visit.log 2>&1 || { echo visit tests failed; exit 1; }
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/l_suite.log 2>&1 || { echo suite failed; tail -30 gpurun_out/l_suite.log; exit 1; }
tail -3 gpurun_out/l_suite.log
timeout -k 10 300 python3 bench.py > gpurun_out/l_bench.log 2>&1 || { echo bench failed; exit 1; }
tail -1 gpurun_out/l_bench.log | cut -c1-400
