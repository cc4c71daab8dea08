#!/bin/bash
# PMC counter passes of the driver's command (tools/gpu_pmc.sh), its rocprofv3 kernel trace, and
# the configs[4]-literal (QMIX 4 x 16) observe A/B: split launches (default) vs one workgroup per
# env (LBSIM_OBSERVE_SPLIT_S=64).  usage: bash tools/gpu_measure2.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-measure2}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/qmix64.jsonl
for rep in 1 2; do
  for v in "LBSIM_OBSERVE_SPLIT_S=16" "LBSIM_OBSERVE_SPLIT_S=64"; do
    echo "== $v rep $rep" >> $O/qmix64.jsonl
    env $v timeout -k 10 240 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 --workload qmix --servers 64 >> $O/qmix64.jsonl 2>> $O/qmix64.err || exit 40
  done
done
for v in "LBSIM_OBSERVE_SPLIT_S=4" "LBSIM_OBSERVE_SPLIT_S=64"; do
  echo "== $v" >> $O/s8.jsonl
  env $v timeout -k 10 240 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 --trace poisson_for_loop_rate_500 --servers 8 >> $O/s8.jsonl 2>> $O/s8.err || exit 41
done
bash tools/gpu_pmc.sh $TAG/pmc || exit 42
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-graph > $O/prof_bench.log 2>&1 || exit 43
