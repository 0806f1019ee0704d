#!/bin/bash
# round-3 GPU call T: per-pivot reciprocal in the windowed panel -- tail microbenchmark A/B, bitwise tests, benches
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 120 ubt_old.log tools/ubench_tail_old 4441 5 || exit 1
$S 120 ubt_new.log tools/ubench_tail 4441 5 || exit 1
$S 120 ubt_old1k.log tools/ubench_tail_old 1024 3 || exit 1
$S 120 ubt_new1k.log tools/ubench_tail 1024 3 || exit 1
$S 400 r03t_panel.log python -u -m pytest tests/test_gpu_panel.py tests/test_gpu_kkt.py -m gpu -x -q --timeout 200 --timeout-method thread -rfEx || exit 1
$S 300 r03t_bench.log python3 bench.py --steps 5 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
$S 200 r03t_bp.log python3 tools/banded_probe.py 3 1 || exit 1
