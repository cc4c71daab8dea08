#!/bin/bash
# observe A/B at the headline shape: the workgroup-per-env observe_kernel (LBSIM_OBSERVE=wg) against
# observe_stream_kernel at 2 / 3 / 4 waves per SIMD, then the driver's exact command with and
# without the scratch-env pre-warm.  usage: bash tools/gpu_obs_ab.sh <tag> [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-obsab}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="python bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 10 $@"
: > $O/ab.jsonl
for v in "LBSIM_OBSERVE=wg" "LBSIM_OBSERVE_OCC=2" "LBSIM_OBSERVE_OCC=3" "LBSIM_OBSERVE_OCC=4" "LBSIM_OBSERVE=wg" "LBSIM_OBSERVE_OCC=2"; do
  echo "== $v" >> $O/ab.jsonl
  env $v timeout -k 10 240 $B >> $O/ab.jsonl 2>> $O/ab.err || exit 20
done
echo "== driver cmd, prewarm 0" >> $O/ab.jsonl
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --prewarm-ms 0 >> $O/ab.jsonl 2>> $O/ab.err || exit 21
echo "== driver cmd, prewarm 200" >> $O/ab.jsonl
timeout -k 10 240 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline >> $O/ab.jsonl 2>> $O/ab.err || exit 22
