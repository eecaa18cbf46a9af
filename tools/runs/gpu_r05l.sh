set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05l
AB_ROUNDS=7 AB_ONLY=park_rec2,rec6,diag_park_rec2_memory,park_round4 timeout -k 10 150 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 3
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu > ${P}_cfg4.json 2> ${P}_cfg4.err || exit 4
