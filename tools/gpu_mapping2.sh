#!/bin/bash
# Mapping sweep (env-per-lane vs server-per-lane dynamics) over batch sizes and server counts.
# usage: bash tools/gpu_mapping2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-mapping}
mkdir -p $O
cd $R
: > $O/sweep.jsonl
for cfg in "--batch 16384" "--batch 32768" "--batch 65536" "--batch 131072" "--batch 16384 --servers 8" "--batch 65536 --servers 8" "--batch 65536 --servers 8 --trace poisson_for_loop_rate_500" "--batch 8192 --servers 16"; do
  for m in env server; do
    echo "{\"variant\": \"$m\", \"round\": 1, \"args\": \"$cfg\"}" >> $O/sweep.jsonl
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --dyn-mapping $m $cfg >> $O/sweep.jsonl 2>> $O/err.log || exit 12
  done
done
