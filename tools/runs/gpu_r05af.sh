set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05af
T="--timeout 150 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_blocksums.py -m gpu -x -q $T -k "past_4gib or lpark or variants" > ${P}_pytest.log 2>&1 || { tail -40 ${P}_pytest.log; exit 3; }
AB_ROUNDS=3 AB_ONLY=lpark,park_rec2_coalesced,diag_park_rec2_memory timeout -k 10 150 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
SWEEP_SHAPES=2,1 SWEEP_ROUNDS=2 timeout -k 10 400 python tools/blocklen_sweep.py > ${P}_sweep.jsonl 2> ${P}_sweep.err || exit 4
