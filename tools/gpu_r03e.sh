#!/bin/bash
# round-3 GPU call E: the GPU test suite and the bench
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 850 r03e_pytest.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfEx || exit 1
$S 280 r03e_bench.log python -u bench.py --steps 10 --warmup 2 || exit 1
