#!/bin/bash
# tests + smoke + bench + split/fused A/B + kernel trace (gpu_r03.sh), then the PMC passes and the
# VALU micro-benchmark (gpu_pmc_r03.sh).  usage: bash tools/gpu_r03c.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r03c}
bash $R/tools/gpu_r03.sh $TAG || exit $?
bash $R/tools/gpu_pmc_r03.sh ${TAG}_pmc || exit $?
