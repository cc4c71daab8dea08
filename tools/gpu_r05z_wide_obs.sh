set -o pipefail
mkdir -p gpurun_out/r05z
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_multi_agent_gpu.py -m gpu > gpurun_out/r05z/tests.txt 2>&1 || exit 11
bash tools/gpu_lib_ab.sh r05z/qmix cur cur:LBSIM_OBSERVE_PAIRED=0 p16w3 -- --workload qmix --steps 30 --warmup 5 || exit 12
bash tools/gpu_lib_ab.sh r05z/qmix64 cur cur:LBSIM_OBSERVE_PAIRED=0 -- --workload qmix --servers 64 --steps 30 --warmup 5 || exit 13
