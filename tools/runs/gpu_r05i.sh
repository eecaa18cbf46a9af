# round-5 GPU step i: read+write stream diagnostics (record write bursts)
set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05i
timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
