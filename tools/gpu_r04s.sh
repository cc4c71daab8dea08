#!/bin/bash
# S = 5-8 one-launch step at 2-4 envs per SIMD: the parity / dispatch tests that cover it, then
# the base library (HEAD before the change) against the current one at 4096 x 8, 2048 x 8,
# 3072 x 6 and 4096 x 4, twice each in alternating order.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04s}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "dispatch or occupancy or configs1 or simulator_bit_exact or wave_kernel" \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
for shape in "--batch 4096 --servers 8" "--batch 2048 --servers 8" "--batch 3072 --servers 6" "--batch 4096 --servers 4"; do
  n=$(echo $shape | tr -d ' -')
  bash $R/tools/gpu_lib_ab.sh $TAG/$n base cur -- --steps 30 --warmup 5 $shape || exit 11
done
