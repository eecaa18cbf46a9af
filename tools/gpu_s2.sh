set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_filesums.py tests/test_gpu_large.py tests/test_c_abi.py -x -v --timeout 200 --timeout-method thread > gpurun_out/s2_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload filesums > gpurun_out/s2_filesums.json 2> gpurun_out/s2_filesums.err || exit 1
RSG_FILESUMS_KERNEL=0 timeout -k 10 300 python bench.py --workload filesums --cpu-seconds 1 > gpurun_out/s2_filesums_ring.json 2> gpurun_out/s2_filesums_ring.err || exit 1
