set -o pipefail
mkdir -p gpurun_out
echo ab; timeout -k 10 300 python bench.py --ab --steps 30 --windows 1 --no-cpu --no-host-path --no-delivery > gpurun_out/s8_ab.json 2>gpurun_out/s8_ab.err || exit 1
echo tests; timeout -k 10 300 python -u -m pytest tests/test_gpu_blocksums.py tests/test_gpu_filesums.py -x -q -m gpu -k "variants_device_aligned or kernel_variants or filesums" --timeout 200 --timeout-method thread > gpurun_out/s8_pytest.log 2>&1 || exit 1
echo cfg4; RSG_BLOCKSUMS_KERNEL=7 timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-delivery > gpurun_out/s8_cfg4_k7.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-delivery > gpurun_out/s8_cfg4_k2.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --workload filesums --cpu-seconds 0.5 > gpurun_out/s8_filesums.json 2>gpurun_out/s8_filesums.err || exit 1
