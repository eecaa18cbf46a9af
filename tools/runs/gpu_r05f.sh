# round-5 GPU step f: park with coalesced record stores (A/B), cfg3 speculative
# selection with O(n) chaining vs the whole-range batch
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/r05f
timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
for r in 1 2; do
timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_spec$r.json 2> ${P}_cfg3_spec$r.err || exit 3
RSG_CONFIRM_SPEC=0 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_nospec$r.json 2> ${P}_cfg3_nospec$r.err || exit 4
done
