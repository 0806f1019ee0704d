#!/bin/bash
# round-3 GPU call H: tail look-ahead inside the per-phase redo, redo counters, factor tests, bench
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 120 ubt3_4441.log tools/ubench_tail 4441 5 || exit 1
$S 120 ubt3_1024.log tools/ubench_tail 1024 3 || exit 1
$S 200 rs_new4.log python3 tools/redo_stats.py linear-programming-vanderbei_amd 2 || exit 1
$S 400 r03j_kkt.log python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_panel.py -m gpu -q --timeout 300 --timeout-method thread -rfEx || exit 1
$S 300 r03j_bench.log python3 bench.py --steps 10 --warmup 2 --cpu-iters 0 --block-angular off --hbm off --banded off || exit 1
