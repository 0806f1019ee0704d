#!/bin/bash
# round-3 GPU call C: widened dense tail (default rho 0.7): sweeps, GPU tests, bench
mkdir -p gpurun_out
S=tools/gpu_step.sh
for meth in hsd intpt hsdls; do
  SWEEP_SAVE=gpurun_out/sweep_rho07 SWEEP_METHOD=$meth SWEEP_SKIP=pds-06 \
    $S 400 r03c_sweep_$meth.log python -u tools/gpu_sweep.py || exit 1
done
$S 900 r03c_pytest.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfEx || exit 1
$S 600 r03c_bench.log python -u bench.py --steps 10 --warmup 2 || exit 1
