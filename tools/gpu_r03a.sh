#!/bin/bash
# round-3 GPU call A: GPU tests, bench, dependent-pivot dumps, trace sweep, config3 probe
mkdir -p gpurun_out
S=tools/gpu_step.sh
$S 900 r03a_pytest.log python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rfEx || exit 1
$S 300 r03a_dumps.log python -u tools/gpu_dump.py gpurun_out/dumps stocfor2 agg2 bandm share1b agg3 lotfi:intpt lotfi:hsdls blend:intpt || exit 1
$S 600 r03a_bench.log python -u bench.py --steps 5 --warmup 1 || exit 1
SWEEP_SAVE=gpurun_out/sweep SWEEP_SKIP=dfl001 $S 600 r03a_sweep.log python -u tools/gpu_sweep.py || exit 1
$S 400 r03a_config3.log python -u tools/synth_run.py random 200000 1000000 256 || exit 1
