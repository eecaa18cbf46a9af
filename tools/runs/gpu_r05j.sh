set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05j
AB_ROUNDS=7 AB_ONLY=park,stream_rw,stream_3w_park,no_records timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
export TMPDIR=/tmp
mkdir -p ${P}_trace_nospec ${P}_trace_spec
RSG_CONFIRM_SPEC=0 timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d ${P}_trace_nospec -o trace -- python3 bench.py --workload cfg3 --steps 2 --warmup 1 --no-cpu --no-host-path > ${P}_trace_nospec.log 2>&1 || exit 3
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d ${P}_trace_spec -o trace -- python3 bench.py --workload cfg3 --steps 2 --warmup 1 --no-cpu --no-host-path > ${P}_trace_spec.log 2>&1 || exit 4
