set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05ac
T="--timeout 150 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocksums.py -m gpu -x -q $T -k "variants" > ${P}_pytest.log 2>&1 || { tail -40 ${P}_pytest.log; exit 2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q $T -k "past_4gib" > ${P}_pytest_large.log 2>&1 || { tail -40 ${P}_pytest_large.log; exit 3; }
SWEEP_SHAPES=2,1,0,4 SWEEP_ROUNDS=2 timeout -k 10 400 python tools/blocklen_sweep.py > ${P}_sweep.jsonl 2> ${P}_sweep.err || exit 4
