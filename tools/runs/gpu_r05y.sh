set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05y
SWEEP_SHAPES=2 SWEEP_ROUNDS=3 timeout -k 10 300 python tools/blocklen_sweep.py > ${P}_sweep.jsonl 2> ${P}_sweep.err || exit 4
