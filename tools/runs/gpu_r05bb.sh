set -o pipefail
cd $GRAFT_REPO_ROOT
SWEEP_BLENS=9216,12288,16384,20480,24576,32768 SWEEP_ROUNDS=2 SWEEP_ONLY=automatic,staged,staged_seg128,staged_seg128_persist,pipe_seg512 \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/r05bb_sweep.jsonl 2> gpurun_out/r05bb_sweep.err || exit 4
