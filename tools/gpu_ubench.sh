#!/bin/bash
# Micro-benchmarks + single-env kernel trace.  usage: bash tools/gpu_ubench.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-ubench}
mkdir -p $O
cd $R
timeout -k 10 120 ./tools/ubench_mul > $O/ubench_mul.json 2> $O/ubench_err.log || exit 10
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_single -o single --output-format csv -- python3 $R/tools/single_env_latency.py --steps 300 > $O/single_prof.log 2>&1 || exit 11
