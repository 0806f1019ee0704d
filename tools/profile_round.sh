#!/bin/bash
# Round profile on the GPU box (developer tool):
#   1. bench.py, default flags                 -> gpurun_out/<tag>_bench.log
#   2. rocprofv3 --kernel-trace --stats, same  -> gpurun_out/<tag>_trace/
#   3. two PMC passes (FETCH_SIZE, WRITE_SIZE) on one complete solve
tag=${1:-r01}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/${tag}_bench.log 2>&1 || exit 1
# rocprofv3 has been seen to fault in its own finalisation after writing the
# database (cooperative launches in the trace): go on when the database exists
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${tag}_trace -o run -- python3 bench.py --steps 2 --warmup 0 --block-angular off --hbm off > gpurun_out/${tag}_trace.log 2>&1 || test -s gpurun_out/${tag}_trace/run_results.db || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/${tag}_pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-iters 0 --no-timing --block-angular off --hbm off > gpurun_out/${tag}_pmc_fetch.log 2>&1 || test -s gpurun_out/${tag}_pmc_fetch/run_results.db || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/${tag}_pmc_write -o run -- python3 bench.py --steps 1 --warmup 0 --cpu-iters 0 --no-timing --block-angular off --hbm off > gpurun_out/${tag}_pmc_write.log 2>&1 || test -s gpurun_out/${tag}_pmc_write/run_results.db || exit 1
