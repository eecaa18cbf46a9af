set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05ag
T="--timeout 150 --timeout-method thread"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q $T > ${P}_pytest.log 2>&1 || { tail -40 ${P}_pytest.log; exit 2; }
SWEEP_SHAPES=2,4,1 SWEEP_ROUNDS=2 timeout -k 10 400 python tools/blocklen_sweep.py > ${P}_sweep.jsonl 2> ${P}_sweep.err || exit 4
