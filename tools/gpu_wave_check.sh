set -o pipefail
O=gpurun_out/${1:-w1}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "simulator_bit_exact or wave_kernel" > $O/pytest.log 2>&1; echo "pytest rc=$?" >> $O/pytest.log
for w in 1 0; do
  LBSIM_DYN_WAVE=$w timeout -k 10 200 python bench.py --no-cpu-baseline --no-graph --steps 30 --warmup 5 --batch 4096 >> $O/bench_4096.jsonl 2>> $O/err.log || exit 12
done
for w in 1 0; do
  LBSIM_DYN_WAVE=$w timeout -k 10 200 python tools/single_env_latency.py --steps 1000 >> $O/latency.jsonl 2>> $O/err.log || exit 13
done
timeout -k 10 200 python tools/single_env_breakdown.py --steps 1000 > $O/breakdown.json 2>> $O/err.log || exit 14
