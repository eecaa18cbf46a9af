set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blocksums.py -m gpu -x -q --timeout 200 --timeout-method thread -k "7 or sqrt or automatic" > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
SWEEP_SQRT=1 SWEEP_ONLY=automatic,lines timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sqrt.jsonl 2> gpurun_out/${T}_sqrt.err || { tail -20 gpurun_out/${T}_sqrt.err; exit 7; }
cut -c1-300 gpurun_out/${T}_sqrt.jsonl
