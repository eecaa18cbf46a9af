set -o pipefail
cd $GRAFT_REPO_ROOT
T=r05ax
bash tools/gpu_run.sh $T tests smoke bench || exit 1
SWEEP_BLENS=9000,10000,12000,16000,20000,24000,24576,28000 SWEEP_ONLY=automatic,staged,staged_seg128,pipe_seg512 \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep.jsonl 2> gpurun_out/${T}_sweep.err || exit 4
