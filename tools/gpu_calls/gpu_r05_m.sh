#!/bin/bash
# round-5 GPU call m: threaded ordering -- host setup split per thread
# count (IPO_HIP_SETUP_TIMES), the symbolic tests, then the bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
nproc > gpurun_out/m_setup.log
for t in 1 4 8 16; do
  echo "threads $t" >> gpurun_out/m_setup.log
  IPO_HIP_SETUP_THREADS=$t IPO_HIP_SETUP_TIMES=1 timeout -k 10 120 python3 -c "
import sys, time; sys.path[:0]=['linear-programming-vanderbei_amd','tests']
import ipo_amd; from conftest import mps_path
p = ipo_amd.load_mps(mps_path('dfl001'))
for r in range(3):
    t=time.time(); s=ipo_amd.symbolic(p.m, p.n, p.kA, p.iA); print('symbolic %.1f ms' % (1e3*(time.time()-t)), flush=True)
" >> gpurun_out/m_setup.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -m pytest -x -q tests/test_symbolic.py > gpurun_out/m_sym.log 2>&1 || { echo sym failed; exit 1; }
timeout -k 10 300 python3 bench.py > gpurun_out/m_bench.log 2>&1 || { echo bench failed; exit 1; }
cat gpurun_out/m_setup.log
tail -1 gpurun_out/m_bench.log | grep -o '"end_to_end[^}]*}'
