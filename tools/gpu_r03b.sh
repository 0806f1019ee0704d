#!/bin/bash
# round-3 GPU call B: zero-pivot rule sweeps (IPO_HIP_PIVTOL) and dense-tail width A/B
mkdir -p gpurun_out
S=tools/gpu_step.sh
for tau in 0 1e-17; do
  for meth in hsd intpt hsdls; do
    SWEEP_SAVE=gpurun_out/sweep_tau$tau SWEEP_METHOD=$meth SWEEP_SKIP=dfl001,pds-06 IPO_HIP_PIVTOL=$tau \
      $S 400 r03b_sweep_${tau}_$meth.log python -u tools/gpu_sweep.py || exit 1
  done
done
DFL=$(python -c "import sys;sys.path.insert(0,'tests');from conftest import mps_path;print(mps_path('dfl001'))")
IPO_HIP_PIVTOL=0 $S 200 r03b_dfl001_tau0.log linear-programming-vanderbei_amd/bin/ipo_hip $DFL hsd --no-out || exit 1
$S 600 r03b_rho.log bash tools/gpu_rho.sh || exit 1
