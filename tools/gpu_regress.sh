#!/bin/bash
# Same-box regression check: the round-2 tree (expl/r02, built in-tree) vs this tree, headline
# bench interleaved.
set -o pipefail
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:-regress}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_multi_agent_gpu.py tests/test_env_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || exit 10
: > $O/ab.jsonl
for r in 1 2 3; do
  for v in r02 r03; do
    echo "{\"variant\": \"$v\", \"round\": $r, \"args\": \"--batch 65536\"}" >> $O/ab.jsonl
    case $v in
      r02) cd $R/expl/r02; X="" ;;
      r03) cd $R; X=--no-graph ;;
    esac
    timeout -k 10 240 python bench.py --no-cpu-baseline --steps 50 --warmup 10 $X >> $O/ab.jsonl 2>> $O/err.log || exit 12
  done
done
