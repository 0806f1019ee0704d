cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash tools/gpu_step.sh 300 trace0.log rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace0 -o run -- python3 bench.py --steps 30 --warmup 1 --cpu-iters 0 --no-timing --block-angular off || exit 1
bash tools/gpu_step.sh 200 bench0.log python3 bench.py --cpu-iters 0 --block-angular off --no-timing || exit 1
