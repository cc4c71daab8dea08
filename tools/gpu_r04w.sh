#!/bin/bash
# PMC passes of the one-launch step at configs[1]'s 4096 x 4 and at 4096 x 8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
bash $R/tools/gpu_pmc.sh r04w/s4 --batch 4096 || exit 11
bash $R/tools/gpu_pmc.sh r04w/s8 --batch 4096 --servers 8 || exit 12
