#!/bin/bash
# Wave (one wave per env) vs group (server-per-lane) dynamics across batch sizes, S = 4:
# usage: bash tools/gpu_wave_sweep.sh <tag> [extra bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-wsweep}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for b in 1024 2048 4096 8192 16384 32768; do
  for w in 1 0; do
    echo "B=$b wave=$w" >> $O/progress.log
    LBSIM_DYN_WAVE=$w timeout -k 10 200 python bench.py --no-cpu-baseline --no-graph --steps 20 --warmup 3 --batch $b "$@" >> $O/sweep_w$w.jsonl 2>> $O/err.log || exit 12
  done
done
