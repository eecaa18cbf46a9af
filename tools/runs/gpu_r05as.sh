set -o pipefail
cd $GRAFT_REPO_ROOT
SWEEP_BLENS=776,832,904,960,1100,1152,1280,9000,10000,12000,16000,20000,24000,32000 SWEEP_ONLY=automatic,staged,staged_seg128,pipe_seg512,pipe \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/r05as_sweep.jsonl 2> gpurun_out/r05as_sweep.err || exit 4
