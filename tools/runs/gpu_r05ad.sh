set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05ad
AB_ROUNDS=3 AB_ONLY=lpark,diag_park_memory_only,park_rec2_coalesced,diag_park_rec2_memory timeout -k 10 150 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
