#!/bin/bash
# round-3 GPU call F: dense-tail microbenchmark, then the round profile
mkdir -p gpurun_out
timeout -k 10 120 tools/ubench_tail 4441 5 > gpurun_out/ubt_4441.log 2>&1 || exit 1
timeout -k 10 120 tools/ubench_tail 1024 3 > gpurun_out/ubt_1024.log 2>&1 || exit 1
timeout -k 10 120 tools/ubench_tail_st 4441 1 60 > gpurun_out/ubt_st60.log 2>&1 || exit 1
timeout -k 10 120 tools/ubench_tail_st 4441 1 2 > gpurun_out/ubt_st2.log 2>&1 || exit 1
bash tools/profile_round.sh r03
