#!/bin/bash
# Round-6 session pass: every GPU test and smoke(), then A/Bs of the headline (library builds
# and auto-reset modes, two alternating rounds), then the driver's bench command.
# usage: bash tools/gpu_r06.sh <tag> [lib variants for gpu_lib_ab.sh, default "base cur"]
#   SKIP_TESTS=1: no pytest / smoke;  MODES="<variants>": the next-step A/B of these variants
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r06}; shift
VARS=${@:-base cur}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
fi
bash tools/gpu_lib_ab.sh $TAG/ab $VARS -- || exit 12
bash tools/gpu_lib_ab.sh $TAG/modes ${MODES:-cur} -- --autoreset-mode next_step || exit 13
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_cmd.json 2> $O/bench.err || exit 14
