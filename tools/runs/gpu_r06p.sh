set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06p
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blocksums.py tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -2 gpurun_out/${T}_t1.log
SWEEP_SQRT=1 SWEEP_ONLY=automatic timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sqrt.jsonl 2> gpurun_out/${T}_sqrt.err || { tail -20 gpurun_out/${T}_sqrt.err; exit 7; }
cut -c1-220 gpurun_out/${T}_sqrt.jsonl
timeout -k 10 300 python bench.py --workload cfg3 --no-host-path > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
cut -c1-300 gpurun_out/${T}_cfg3.json
