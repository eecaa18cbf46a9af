set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_filesums.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/s4_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload filesums --cpu-seconds 1 > gpurun_out/s4_filesums.json 2> gpurun_out/s4_filesums.err || exit 1
timeout -k 10 300 python bench.py --workload cfg3 --cpu-seconds 1 > gpurun_out/s4_cfg3.json 2> gpurun_out/s4_cfg3.err || exit 1
RSG_ROLL_KERNEL=0 timeout -k 10 300 python bench.py --workload cfg3 --no-cpu > gpurun_out/s4_cfg3_old.json 2> gpurun_out/s4_cfg3_old.err || exit 1
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --cpu-seconds 1 > gpurun_out/s4_cfg4.json 2> gpurun_out/s4_cfg4.err || exit 1
