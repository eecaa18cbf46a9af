set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/s5_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload cfg3 --cpu-seconds 1 > gpurun_out/s5_cfg3.json 2> gpurun_out/s5_cfg3.err || exit 1
RSG_ROLL_KERNEL=0 timeout -k 10 300 python bench.py --workload cfg3 --no-cpu > gpurun_out/s5_cfg3_old.json 2> gpurun_out/s5_cfg3_old.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --no-host-path --steps 20 > gpurun_out/s5_cfg2.json 2> gpurun_out/s5_cfg2.err || exit 1
