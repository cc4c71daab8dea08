#!/bin/bash
# tests + smoke, then the headline A/B: current build at 16 (default), 13 and 12 envs per
# dynamics wave (LBSIM_DYN_EPW), and the round-start library r04f.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04k}
bash $R/tools/gpu_tests.sh $TAG || exit $?
bash $R/tools/gpu_lib_ab.sh $TAG cur cur:LBSIM_DYN_EPW=13 cur:LBSIM_DYN_EPW=12 r04f || exit $?
