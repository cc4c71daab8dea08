#!/bin/bash
# Measurement pass of the headline: pre-warm A/B, the PMC counter passes (tools/gpu_pmc.sh) and a
# rocprofv3 kernel trace of the driver's command.  usage: bash tools/gpu_measure.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-measure}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
bash tools/gpu_prewarm_ab.sh $TAG || exit 31
bash tools/gpu_pmc.sh $TAG/pmc || exit 32
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-graph > $O/prof_bench.log 2>&1 || exit 33
