set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06e
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_sender_small.py tests/test_gpu_filesums.py tests/test_gpu_blocksums.py tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
for r in 1 2; do
  RSG_LIB_PATH=rsync_amd/ab/librsg_r05.so timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-path --no-delivery > gpurun_out/${T}_cfg2_old$r.json 2> gpurun_out/${T}_cfg2_old$r.err || exit 2
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-path --no-delivery > gpurun_out/${T}_cfg2_new$r.json 2> gpurun_out/${T}_cfg2_new$r.err || exit 3
done
timeout -k 10 400 python bench.py --workload cfg4-sender --steps 10 --cpu-seconds 5 > gpurun_out/${T}_cfg4s.json 2> gpurun_out/${T}_cfg4s.err || { tail -20 gpurun_out/${T}_cfg4s.err; exit 4; }
timeout -k 10 300 python bench.py --workload filesums > gpurun_out/${T}_filesums.json 2> gpurun_out/${T}_filesums.err || { tail -20 gpurun_out/${T}_filesums.err; exit 5; }
timeout -k 10 300 python bench.py --workload cfg3 --no-host-path > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
