#!/bin/bash
# Knob A/Bs on the current library: 8-lane groups at the headline (4 servers: lanes 4-7 only draw
# arrivals ahead), and the OCC-2 one-launch form at 4 envs per SIMD (4096 x 4, 4096 x 8).
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-r04u}
bash $R/tools/gpu_lib_ab.sh $TAG/head cur cur:LBSIM_DYN_GROUP_LANES=8 -- --steps 50 --warmup 10 || exit 11
bash $R/tools/gpu_lib_ab.sh $TAG/b4096s4 cur cur:LBSIM_STEP_WAVE_OCC=2 -- --steps 30 --warmup 5 --batch 4096 || exit 12
bash $R/tools/gpu_lib_ab.sh $TAG/b4096s8 cur cur:LBSIM_STEP_WAVE_OCC=2 -- --steps 30 --warmup 5 --batch 4096 --servers 8 || exit 13
