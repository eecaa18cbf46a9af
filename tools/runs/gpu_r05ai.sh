set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05ai
AB_ROUNDS=7 AB_ONLY=park_rec2_coalesced,diag_park_rec2_memory,rec7 timeout -k 10 200 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
