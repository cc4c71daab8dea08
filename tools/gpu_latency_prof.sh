#!/bin/bash
# The single-env drop-in step (tools/single_env_latency.py, B = 1): the single-env tests, us/step
# at the default group width and forced 4 / 16 lanes, and a kernel trace (per-launch durations vs
# the measured us/step).  usage: bash tools/gpu_latency_prof.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-latprof}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_env_gpu.py tests/test_plumbing.py -x -q -m gpu --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 10
timeout -k 10 300 python tools/single_env_latency.py --steps 2000 > $O/latency.jsonl 2>> $O/err.log || exit 11
for g in 4 16; do
  LBSIM_DYN_GROUP_LANES=$g timeout -k 10 300 python tools/single_env_latency.py --steps 2000 >> $O/latency.jsonl 2>> $O/err.log || exit 12
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o lat --output-format csv -- python3 $R/tools/single_env_latency.py --steps 500 > $O/lat.log 2>&1 || exit 14
