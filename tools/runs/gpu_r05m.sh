set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05m
AB_ROUNDS=7 AB_ONLY=park_rec2,rec6,diag_park_rec2_memory,park_round4 timeout -k 10 150 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
for r in 1 2 3; do
  RSG_LIB_PATH=rsync_amd/ab/librsg_rollbase.so timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_base$r.json 2> ${P}_cfg3_base$r.err || exit 3
  timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_new$r.json 2> ${P}_cfg3_new$r.err || exit 4
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 5
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu > ${P}_cfg4.json 2> ${P}_cfg4.err || exit 6
