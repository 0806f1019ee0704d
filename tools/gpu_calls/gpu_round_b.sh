#!/bin/bash
# quick GPU check: KKT parity tests, the dfl001 headline test, a kernel trace and the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
tag=${1:-b}
bash tools/gpu_step.sh 400 tests_$tag.log python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_kkt.py "tests/test_gpu_ipm.py::test_dfl001_hsd_headline" -m gpu || exit 1
grep -q "passed" gpurun_out/tests_$tag.log && ! grep -q "failed" gpurun_out/tests_$tag.log || exit 1
bash tools/gpu_step.sh 300 trace_$tag.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_$tag -o run -- python3 bench.py --steps 30 --warmup 1 --cpu-iters 0 --no-timing --block-angular off || exit 1
bash tools/gpu_step.sh 200 bench_$tag.log python3 bench.py --cpu-iters 0 --block-angular off --no-timing || exit 1
