#!/bin/bash
# Observe fma change: GPU parity (all simulator / features cases), headline bench x3, then the
# 4k-512k batch sweep with the 2-group async figure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-s5g}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
: > $O/ab.jsonl
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --no-cpu-baseline >> $O/ab.jsonl 2>> $O/ab.err || exit 11
done
bash tools/gpu_sweep.sh ${TAG}_sweep --async-groups 2 || exit 12
