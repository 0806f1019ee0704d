#!/bin/bash
# A/B of KKT kernel variants on dfl001 (developer tool): one short bench per
# setting, env given as NAME=VALUE words; stops at the first failure.
# usage: gpu_ab.sh "<label> VAR=v ..." ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for spec in "$@"; do
    set -- $spec; label=$1; shift
    env "$@" timeout -k 10 200 python3 bench.py --steps 3 --warmup 1 --cpu-iters 0 --block-angular off --hbm off --no-timing > gpurun_out/ab_$label.log 2>&1
    rc=$?
    echo "[$label] rc=$rc $(grep -o '"value": [0-9.a-z]*' gpurun_out/ab_$label.log) $(grep -o '"iterations_per_solve": \[[0-9, ]*\]' gpurun_out/ab_$label.log) $(grep -o '"final_mu": [0-9.e+-]*' gpurun_out/ab_$label.log)" | tee -a gpurun_out/ab.txt
    [ $rc -eq 0 ] || exit 99
done
