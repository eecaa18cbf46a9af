set -o pipefail
cd $GRAFT_REPO_ROOT
T=r05bc
bash tools/gpu_run.sh $T tests smoke bench || exit 1
SWEEP_BLENS=1000,2176,4000,9000,9216,16384,24576,32768 SWEEP_ONLY=automatic,staged,staged_seg128,pipe_seg512 \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep.jsonl 2> gpurun_out/${T}_sweep.err || exit 4
SWEEP_ONLY=automatic timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep_pow2.jsonl 2> gpurun_out/${T}_sweep_pow2.err || exit 5
