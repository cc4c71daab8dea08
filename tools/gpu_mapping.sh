#!/bin/bash
# Dynamics mapping study: simulator parity under both mappings, then bench each mapping over the
# batch / server-count grid of BASELINE configs (one JSON line per run in $O/sweep.jsonl).
# usage: bash tools/gpu_mapping.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-map}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -q -x -k simulator > $O/pytest_parity.log 2>&1 || exit 10
: > $O/sweep.jsonl
run() {
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 30 --warmup 5 "$@" >> $O/sweep.jsonl 2> $O/last_err.log || exit 12
}
for m in env server; do
  for b in 4096 8192 16384 32768 65536; do run --batch $b --servers 4 --dyn-mapping $m; done
  run --batch 8192 --servers 8 --dyn-mapping $m
  run --batch 65536 --servers 8 --dyn-mapping $m
  run --workload qmix --batch 8192 --servers 16 --dyn-mapping $m
done
