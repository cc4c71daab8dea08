#!/bin/bash
# tests + smoke, library A/B at the headline, the default bench line (graph leg included).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04i}
O=$R/gpurun_out/$TAG
bash $R/tools/gpu_tests.sh $TAG || exit $?
bash $R/tools/gpu_lib_ab.sh $TAG cur r04f || exit $?
cd $R
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit 12
