set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06ae
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sender_small.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -3 gpurun_out/${T}_t1.log
