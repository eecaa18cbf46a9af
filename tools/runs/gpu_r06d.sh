set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06d
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sender_small.py tests/test_gpu_filesums.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_small.log 2>&1 || { tail -40 gpurun_out/${T}_small.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_sender_fd.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_match.log 2>&1 || { tail -40 gpurun_out/${T}_match.log; exit 2; }
timeout -k 10 400 python bench.py --workload cfg4-sender --steps 10 --cpu-seconds 5 > gpurun_out/${T}_cfg4s.json 2> gpurun_out/${T}_cfg4s.err || { tail -20 gpurun_out/${T}_cfg4s.err; exit 3; }
timeout -k 10 300 python bench.py --workload filesums > gpurun_out/${T}_filesums.json 2> gpurun_out/${T}_filesums.err || { tail -20 gpurun_out/${T}_filesums.err; exit 4; }
