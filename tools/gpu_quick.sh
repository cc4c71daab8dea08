#!/bin/bash
# Quick GPU pass: simulator parity (both mappings) + bench lines for the given configs.
# usage: bash tools/gpu_quick.sh <tag> "<bench args 1>" "<bench args 2>" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-quick}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -x > $O/pytest_parity.log 2>&1 || exit 10
: > $O/sweep.jsonl
for a in "$@"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $a >> $O/sweep.jsonl 2> $O/last_err.log || exit 12
done
