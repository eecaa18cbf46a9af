set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_blocksums.py -x -v --timeout 200 --timeout-method thread > gpurun_out/s1_pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu > gpurun_out/s1_cfg4.json 2> gpurun_out/s1_cfg4.err || exit 1
timeout -k 10 200 python bench.py --workload cfg5 --steps 20 --no-cpu > gpurun_out/s1_cfg5.json 2> gpurun_out/s1_cfg5.err || exit 1
timeout -k 10 200 python bench.py --no-cpu --no-host-path > gpurun_out/s1_cfg2.json 2> gpurun_out/s1_cfg2.err || exit 1
