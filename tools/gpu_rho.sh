#!/bin/bash
# dense-tail width A/B on dfl001 (IPO_HIP_TAIL_DENSITY), 3 solves each, + traces
mkdir -p gpurun_out
for rho in 1.0 0.9 0.8 0.75 0.7 0.6; do
  IPO_HIP_TAIL_DENSITY=$rho timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --cpu-iters 0 --hbm off --block-angular off > gpurun_out/rho_$rho.json 2> gpurun_out/rho_$rho.err
  rc=$?; echo "rho $rho rc $rc"; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 99; fi
  python -c "import json;d=json.load(open('gpurun_out/rho_$rho.json'));c=d['config'];print('$rho',d['value'],c['iterations_per_solve'],c['final_mu'],c['factor_ms_total'],c['solve_ms_total'],c['setup_s'],d['roofline']['phase'] if d['roofline'] else None)"
done
