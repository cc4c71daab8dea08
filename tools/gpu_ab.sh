#!/bin/bash
# Same-box A/B over several bench configurations: every variant library
# marllb_amd/exp/liblbsim_<name>.so (`python -m marllb_amd.build --variant <name> -D...`; "base" =
# the in-tree marllb_amd/liblbsim.so), loaded through LBSIM_LIBRARY, is first checked by the
# simulator parity tests (PARITY=0 skips) and then benched on every configuration in CONFIGS
# (';'-separated bench argument lists), interleaved over ROUNDS rounds so drift between rounds does
# not favour one variant.
# usage: ROUNDS=2 CONFIGS="--batch 65536;--batch 4096" bash tools/gpu_ab.sh <tag> <name> [<name> ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
TAG=${1:-ab}; shift
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
lib() { if [ "$1" = base ]; then echo $R/marllb_amd/liblbsim.so; else echo $R/marllb_amd/exp/liblbsim_$1.so; fi; }
if [ "${PARITY:-1}" = 1 ]; then
  for n in "$@"; do
    [ "$n" = base ] && continue
    LBSIM_LIBRARY=$(lib $n) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/parity_$n.log 2>&1 || exit 11
  done
fi
: > $O/ab.jsonl
IFS=';' read -ra CFG <<< "${CONFIGS:---batch 65536}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for c in "${CFG[@]}"; do
    for n in "$@"; do
      echo "{\"variant\": \"$n\", \"round\": $r, \"args\": \"$c\"}" >> $O/ab.jsonl
      LBSIM_LIBRARY=$(lib $n) timeout -k 10 240 python bench.py --no-cpu-baseline --steps ${STEPS:-30} --warmup 5 $c >> $O/ab.jsonl 2> $O/err_$n.log || exit 12
    done
  done
done
