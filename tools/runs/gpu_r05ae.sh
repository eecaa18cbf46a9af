set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05ae
T="--timeout 150 --timeout-method thread"
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q $T -k "past_4gib or lpark" > ${P}_pytest_large.log 2>&1 || { tail -40 ${P}_pytest_large.log; exit 3; }
AB_ROUNDS=3 AB_ONLY=lpark,diag_park_memory_only,park_rec2_coalesced,diag_park_rec2_memory timeout -k 10 150 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
