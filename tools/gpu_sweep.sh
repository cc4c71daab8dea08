#!/bin/bash
# Batch sweep of the metric's own range on one GPU (BASELINE metric: batch 4k -> 512k): one bench
# line per (servers, batch), per-kernel HIP-event times inside each line.
# usage: bash tools/gpu_sweep.sh <tag> [extra bench args...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-sweep}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/sweep.jsonl
for S in 4 8; do
  for B in 4096 16384 65536 131072 262144 524288; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 3 --batch $B --servers $S "$@" >> $O/sweep.jsonl 2>> $O/sweep_err.log || exit 31
  done
done
