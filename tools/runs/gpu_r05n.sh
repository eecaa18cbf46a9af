set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05n
export TMPDIR=/tmp
BENCH_DELIVERY_DIAG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-path > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 2
BENCH_DELIVERY_DIAG=1 timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-host-path > ${P}_cfg4.json 2> ${P}_cfg4.err || exit 3
RSG_TIMING=1 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d ${P}_trace -o trace -- python3 bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu --no-host-path > ${P}_cfg3_trace.log 2>&1 || exit 4
