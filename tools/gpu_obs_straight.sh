set -o pipefail
O=gpurun_out/${1:-r03o}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/pytest.log; [ $rc -eq 0 ] || exit 11
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 --batch 4096 >> $O/bench_4096.jsonl 2>> $O/err.log || exit 12
done
for b in 1024 2048; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 --batch $b >> $O/bench_small.jsonl 2>> $O/err.log || exit 13
done
timeout -k 10 200 python tools/single_env_breakdown.py --steps 1000 > $O/breakdown.json 2>> $O/err.log || exit 14
