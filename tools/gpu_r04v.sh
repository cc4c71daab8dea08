#!/bin/bash
# Graph-leg A/B over the HIP runtime's graph submission settings (the eager line alongside).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04v}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/ab.jsonl
for rep in 1 2; do
  for v in "" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=1" "DEBUG_CLR_GRAPH_PACKET_CAPTURE=0" "DEBUG_HIP_GRAPH_BATCH_SIZE=16"; do
    echo "== [$v] rep $rep" >> $O/ab.jsonl
    env $v timeout -k 10 240 python bench.py --no-cpu-baseline --steps 50 --warmup 10 >> $O/ab.jsonl 2>> $O/ab.err || exit 20
  done
done
