#!/bin/bash
# A/B of library builds at the headline shape (marllb_amd/exp/liblbsim_<name>.so through
# LBSIM_LIBRARY; "cur" = the in-tree build), each with optional env settings, twice in
# alternating order.  usage: bash tools/gpu_lib_ab.sh <tag> "<name>[:VAR=val,...]" ... -- [bench args]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=$1; shift
V=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do V+=("$1"); shift; done
[ "$1" == "--" ] && shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
: > $O/ab.jsonl
for rep in 1 2; do
  for v in "${V[@]}"; do
    name=${v%%:*}; envs=""
    [[ "$v" == *:* ]] && envs=$(echo "${v#*:}" | tr ',' ' ')
    lib=""
    [ "$name" != "cur" ] && lib="LBSIM_LIBRARY=$R/marllb_amd/exp/liblbsim_$name.so"
    echo "== $v rep $rep" >> $O/ab.jsonl
    env $lib $envs timeout -k 10 240 python bench.py --no-cpu-baseline --no-graph --steps 50 --warmup 10 "$@" >> $O/ab.jsonl 2>> $O/ab.err || exit 20
  done
done
