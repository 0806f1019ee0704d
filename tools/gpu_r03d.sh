#!/bin/bash
# round-3 GPU call D: fused-panel launch fix (levels without fused units): factor tests, sweeps at the default tail
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 200 r03d_kkt.log python -u -m pytest tests/test_gpu_kkt.py tests/test_gpu_panel.py -m gpu -q --timeout 150 --timeout-method thread -rfEx || exit 1
for meth in hsd intpt hsdls; do
  SWEEP_SAVE=gpurun_out/sweep_r03d SWEEP_METHOD=$meth SWEEP_SKIP=pds-06 \
    $S 280 r03d_sweep_$meth.log python -u tools/gpu_sweep.py || exit 1
done
