set -o pipefail
cd $GRAFT_REPO_ROOT
SWEEP_BLENS=1000,1224,1448,1800,2000,2504,2896,3000,3504,4000,4088,4112,5000,6000,8000 SWEEP_ONLY=automatic,staged,staged_seg128,staged_seg512,staged_seg128_persist,pipe_seg128,pipe_seg512,pipe \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/r05aq_sweep.jsonl 2> gpurun_out/r05aq_sweep.err || exit 4
