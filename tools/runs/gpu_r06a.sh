set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06a
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${T}_match.log 2>&1 || { tail -30 gpurun_out/${T}_match.log; exit 1; }
bash tools/gpu_run.sh $T cfg3 || exit 2
