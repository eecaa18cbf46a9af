set -o pipefail
mkdir -p gpurun_out
bash tools/profile_kernel.sh r03d_cfg2 block_sums --steps 30 --warmup 100 --windows 1 --no-cpu --no-host-path --no-delivery || exit 1
bash tools/profile_kernel.sh r03d_filesums file_sums --workload filesums --steps 10 --cpu-seconds 0.2 || exit 1
echo diag; for D in 3 4; do RSG_BLOCKSUMS_DIAG=$D timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-delivery > gpurun_out/s6_cfg4_diag$D.json 2>/dev/null || exit 1; done
for D in 1 2; do RSG_BLOCKSUMS_DIAG=$D timeout -k 10 200 python bench.py --workload cfg5 --steps 10 --no-cpu > gpurun_out/s6_cfg5_diag$D.json 2>/dev/null || exit 1; done
echo ab; timeout -k 10 200 python bench.py --ab --steps 30 --windows 1 --no-cpu --no-host-path --no-delivery > gpurun_out/s6_ab.json 2>/dev/null || exit 1
echo match; timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s6_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu > gpurun_out/s6_cfg3.json 2> gpurun_out/s6_cfg3.err || exit 1
