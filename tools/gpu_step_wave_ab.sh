#!/bin/bash
# One-launch wave step (AUTO at <= 2 envs per SIMD) vs the two launches (LBSIM_STEP_KERNEL=split),
# S = 4, and the single-env step both ways.  usage: bash tools/gpu_step_wave_ab.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-swab}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "simulator_bit_exact or wave_kernel or dispatch" > $O/pytest.log 2>&1 || exit 10
for b in 1 256 1024 2048 4096; do
  for k in auto split; do
    LBSIM_STEP_KERNEL=$( [ $k = split ] && echo split || echo "" ) timeout -k 10 200 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 --batch $b >> $O/ab_$k.jsonl 2>> $O/err.log || exit 12
  done
done
timeout -k 10 200 python tools/single_env_latency.py --steps 2000 > $O/latency_auto.json 2>> $O/err.log || exit 13
LBSIM_STEP_KERNEL=split timeout -k 10 200 python tools/single_env_latency.py --steps 2000 > $O/latency_split.json 2>> $O/err.log || exit 14
