#!/bin/bash
# developer tool: intpt traces of a few netlib problems on the GPU (gpurun_out/intpt_<name>.txt)
for p in ${@:-brandy e226 agg lotfi scagr7}; do
  f=$(python -c "import sys; sys.path.insert(0,'tests'); from conftest import mps_path; print(mps_path('$p'))")
  timeout -k 5 60 linear-programming-vanderbei_amd/bin/ipo_hip "$f" intpt > gpurun_out/intpt_$p.txt 2>&1 || exit 1
done
