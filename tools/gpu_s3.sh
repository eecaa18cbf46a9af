set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_filesums.py tests/test_gpu_large.py tests/test_c_abi.py tests/test_dist.py tests/test_gpu_match.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/s3_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload filesums > gpurun_out/s3_filesums.json 2> gpurun_out/s3_filesums.err || exit 1
RSG_FILESUMS_KERNEL=0 timeout -k 10 300 python bench.py --workload filesums --cpu-seconds 1 > gpurun_out/s3_filesums_ring.json 2> gpurun_out/s3_filesums_ring.err || exit 1
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --cpu-seconds 2 > gpurun_out/s3_cfg4.json 2> gpurun_out/s3_cfg4.err || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-host-path > gpurun_out/s3_cfg2.json 2> gpurun_out/s3_cfg2.err || exit 1
