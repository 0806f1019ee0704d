#!/bin/bash
# round-3 GPU call L: flat gather -- banded probe, dfl001 bitwise A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 200 r03m_bp.log python3 tools/banded_probe.py 3 1 || exit 1
IPO_HIP_VISIT_SLOTS=32 $S 200 r03m_bp32.log python3 tools/banded_probe.py 3 1 || exit 1
IPO_HIP_GATHER_FLAT=2 $S 300 r03m_bench_flat2.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
$S 300 r03m_bench.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
