#!/bin/bash
# HBM traffic of the fused policy kernels: FETCH_SIZE / WRITE_SIZE passes (one counter group per
# rocprofv3 run, no trace domains) over short sac-gru and qmix bench runs.
# usage: bash tools/gpu_pmc_policy.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-pmc_policy}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for w in sac-gru qmix; do
  B="$R/bench.py --no-cpu-baseline --steps 6 --warmup 2 --workload $w"
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/${w}_fetch -o run --output-format csv -- python3 $B > $O/${w}_fetch.log 2>&1 &&
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/${w}_write -o run --output-format csv -- python3 $B > $O/${w}_write.log 2>&1 || exit 31
done
