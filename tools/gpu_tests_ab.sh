#!/bin/bash
# pytest -m gpu + smoke(), then an A/B of library builds at the headline shape (tools/gpu_lib_ab.sh).
# usage: bash tools/gpu_tests_ab.sh <tag> "<name>[:VAR=val,...]" ... -- [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
bash $R/tools/gpu_tests.sh $TAG || exit $?
bash $R/tools/gpu_lib_ab.sh $TAG "$@" || exit $?
