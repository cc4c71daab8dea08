#!/bin/bash
# Round-2 GPU pass on the current tree: parity tests + smoke + headline bench + rocprofv3 kernel
# trace (gpu_check.sh), the single-env drop-in step latency, and bench.py's self-launched 2-rank
# path rehearsed on one GPU (gloo for the measurement-only collectives).
# usage: bash tools/gpu_r2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r2}
O=$R/gpurun_out/$TAG
cd $R
bash tools/gpu_check.sh $TAG || exit $?
cd $R
timeout -k 10 300 python tools/single_env_latency.py --steps 2000 > $O/single_env_latency.json 2> $O/single_env_err.log || exit 30
LBSIM_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --batch 16384 \
  --no-cpu-baseline > $O/bench_n2_selflaunch.log 2>&1 || exit 31
