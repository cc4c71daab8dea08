#!/bin/bash
# The group kernel's SED score one iteration ahead: parity of every group-kernel case, then the
# library before it (base) against the current one at the headline, 65536 x 8 and 16384 x 4.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04x}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_dynamics_options.py -k "wider_groups or simulator_bit_exact or configs1 or dispatch or options or lost or fail or next" \
  -p no:cacheprovider > $O/pytest_gpu.log 2>&1 || exit 10
bash $R/tools/gpu_lib_ab.sh $TAG/head base cur -- --steps 50 --warmup 10 || exit 11
bash $R/tools/gpu_lib_ab.sh $TAG/s8 base cur -- --steps 30 --warmup 5 --servers 8 || exit 12
bash $R/tools/gpu_lib_ab.sh $TAG/b16k base cur -- --steps 30 --warmup 5 --batch 16384 || exit 13
