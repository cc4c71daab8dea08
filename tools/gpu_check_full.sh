set -o pipefail
O=gpurun_out/${1:-full}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 10
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 11
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 12
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --batch 4096 > $O/bench_4096.json 2>> $O/bench.err || exit 13
