set -o pipefail
cd $GRAFT_REPO_ROOT
SWEEP_BLENS=1152,1536,2176,2560,3072,3584,5120,6144,8192 SWEEP_ONLY=automatic,staged,staged_seg128,staged_seg128_persist,pipe_seg128,pipe_seg512 \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/r05av_sweep.jsonl 2> gpurun_out/r05av_sweep.err || exit 4
