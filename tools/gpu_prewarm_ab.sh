#!/bin/bash
# The driver's exact bench command with and without the scratch-env pre-warm, beside the long
# command, alternating.  usage: bash tools/gpu_prewarm_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-prewarm}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/prewarm.jsonl
for rep in 1 2; do
  for a in "--steps 20 --warmup 5 --prewarm-ms 0" "--steps 20 --warmup 5 --prewarm-ms 200" "--steps 50 --warmup 10 --prewarm-ms 0" "--steps 50 --warmup 10 --prewarm-ms 200"; do
    echo "== $a rep $rep" >> $O/prewarm.jsonl
    timeout -k 10 240 python bench.py --gpus 1 --no-cpu-baseline --no-graph $a >> $O/prewarm.jsonl 2>> $O/prewarm.err || exit 30
  done
done
