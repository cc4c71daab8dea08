#!/bin/bash
# Rehearse bench.py's multi-rank path on one GPU: 2 ranks via torch.distributed.run, gloo for the
# (measurement-only) collectives.  The driver's real N>1 runs use RCCL, one GPU per rank.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-dist}
mkdir -p $O
cd $R
LBSIM_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 10 --warmup 3 --batch 16384 \
  > $O/bench_n2.log 2>&1
