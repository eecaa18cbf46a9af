set -o pipefail
mkdir -p gpurun_out
echo fs; timeout -k 10 300 python -u -m pytest tests/test_gpu_filesums.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s7_pytest.log 2>&1 || exit 1
for K in 1 2; do echo fs$K; RSG_FILESUMS_KERNEL=$K timeout -k 10 300 python bench.py --workload filesums --cpu-seconds 0.5 > gpurun_out/s7_filesums_k$K.json 2>/dev/null || exit 1; done
echo prof; export TMPDIR=/tmp; timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03e_fs/trace -o trace -- python3 bench.py --workload filesums --steps 10 --cpu-seconds 0.2 > gpurun_out/prof_r03e_fs.log 2>&1 || exit 1
timeout -k 10 -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex file_sums --output-format csv -d gpurun_out/prof_r03e_fs/pmc_FETCH_SIZE -o pmc -- python3 bench.py --workload filesums --steps 10 --cpu-seconds 0.2 > gpurun_out/prof_r03e_fs_pmc.log 2>&1 || exit 1
echo cfg3trace; timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r03e_cfg3/trace -o trace -- python3 bench.py --workload cfg3 --cfg3-files 4 --steps 2 --no-cpu > gpurun_out/prof_r03e_cfg3.log 2>&1 || exit 1
