#!/bin/bash
# round-3 GPU call G: deferred tail visits -- microbenchmark, factor tests, dfl001 bench
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 120 ubt2_4441.log tools/ubench_tail 4441 5 || exit 1
$S 120 ubt2_1024.log tools/ubench_tail 1024 3 || exit 1
$S 400 r03g_kkt.log python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_panel.py -m gpu -q --timeout 300 --timeout-method thread -rfEx || exit 1
$S 300 r03g_bench.log python3 bench.py --steps 10 --warmup 2 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
