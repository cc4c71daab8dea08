#!/bin/bash
# step_streams pass 2: split parity (staggered ranges), then A/B of step_streams 1..4 with
# staggered (default) and concurrent (LBSIM_STEP_STAGGER=0) range dynamics.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-streams2}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x -k "split or step_streams" --timeout 120 --timeout-method thread > $O/pytest_split.log 2>&1 || exit 10
: > $O/ab.jsonl
for rep in 1 2; do
  for k in 1 2 3 4; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 10 --step-streams $k >> $O/ab.jsonl 2>> $O/ab.err || exit 11
  done
  for k in 2 3; do
    LBSIM_STEP_STAGGER=0 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 10 --step-streams $k >> $O/ab.jsonl 2>> $O/ab.err || exit 12
  done
done
for k in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 50 --warmup 10 --servers 8 --trace poisson_for_loop_rate_500 --step-streams $k >> $O/ab.jsonl 2>> $O/ab.err || exit 13
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --batch 262144 --step-streams $k >> $O/ab.jsonl 2>> $O/ab.err || exit 14
done
