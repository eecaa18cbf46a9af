set -o pipefail
mkdir -p gpurun_out
T="--timeout 200 --timeout-method thread"
echo tests; timeout -k 10 600 python -u -m pytest tests/test_gpu_blocksums.py tests/test_gpu_large.py tests/test_gpu_filesums.py tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s9_pytest.log 2>&1 || exit 1
echo cfg2; timeout -k 10 300 python bench.py --no-cpu --no-host-path --no-delivery > gpurun_out/s9_cfg2.json 2>gpurun_out/s9_cfg2.err || exit 1
echo cfg4; timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-delivery > gpurun_out/s9_cfg4.json 2>gpurun_out/s9_cfg4.err || exit 1
echo cfg5; timeout -k 10 300 python bench.py --workload cfg5 --steps 20 --no-cpu --no-delivery > gpurun_out/s9_cfg5.json 2>gpurun_out/s9_cfg5.err || exit 1
echo receive; timeout -k 10 300 python bench.py --workload receive > gpurun_out/s9_receive.json 2>gpurun_out/s9_receive.err || exit 1
echo ab; timeout -k 10 300 python bench.py --ab --steps 30 --windows 1 --no-cpu --no-host-path --no-delivery > gpurun_out/s9_ab.json 2>gpurun_out/s9_ab.err || exit 1
echo cfg4k7; RSG_BLOCKSUMS_KERNEL=7 timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-delivery > gpurun_out/s9_cfg4_k7.json 2>/dev/null || exit 1
echo done2
