set -o pipefail
cd $GRAFT_REPO_ROOT
T=r05aw
bash tools/gpu_run.sh $T tests smoke bench || exit 1
SWEEP_BLENS=1000,1152,1224,2176,3072,4000,4096,5120,6144,8192 SWEEP_ONLY=automatic,staged_seg128,pipe_seg512 \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep.jsonl 2> gpurun_out/${T}_sweep.err || exit 4
