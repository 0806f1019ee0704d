#!/bin/bash
# PMC pass on the dense panel kernels (developer tool)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS --kernel-include-regex "k_trsm|k_diag" -d gpurun_out/pmc_dense -o run -- python3 bench.py --steps 3 --warmup 0 --cpu-iters 0 --no-timing > gpurun_out/pmc_dense.log 2>&1
