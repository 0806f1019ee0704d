#!/bin/bash
# run one GPU step under its own time limit; stop the whole call on a fault/timeout
# usage: gpu_step.sh <seconds> <logname> <command...>
secs=$1; shift; log=$1; shift
mkdir -p gpurun_out
timeout -k 10 "$secs" "$@" > "gpurun_out/$log" 2>&1
rc=$?
echo "[$log] rc=$rc" | tee -a gpurun_out/steps.txt
tail -3 "gpurun_out/$log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "STOP: rc=$rc in $log"; exit 99; fi
exit 0
