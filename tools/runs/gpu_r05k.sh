set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05k
AB_ROUNDS=7 AB_ONLY=park,no_records timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
