set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06ah
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_large.py -k "cfg3" -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -4 gpurun_out/${T}_t1.log
