set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06b
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sender_small.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_small.log 2>&1 || { tail -40 gpurun_out/${T}_small.log; exit 1; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_sender_fd.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_match.log 2>&1 || { tail -40 gpurun_out/${T}_match.log; exit 2; }
