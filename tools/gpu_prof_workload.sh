#!/bin/bash
# rocprofv3 kernel trace of one bench workload.  usage: bash tools/gpu_prof_workload.sh <tag> <bench args...>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-wl}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 20 --warmup 5 "$@" > $O/bench.log 2>&1
