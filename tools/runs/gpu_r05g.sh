# round-5 GPU step g: record-store cache policies (A/B), the walk's extra round trip
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/r05g
timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
RSG_WALK_DEBUG=1 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_dbg.json 2> ${P}_cfg3_dbg.err || exit 3
