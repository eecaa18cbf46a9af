set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05p
BENCH_DELIVERY_DIAG=2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-path > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 2
