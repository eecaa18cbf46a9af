set -o pipefail
cd $GRAFT_REPO_ROOT
T=r05ar
bash tools/gpu_run.sh $T tests smoke bench || exit 1
SWEEP_BLENS=704,760,1000,1224,1448,1800,2000,2048,2504,3000,4000,4096,4112,6000,8000,8200 SWEEP_ROUNDS=2 SWEEP_ONLY=automatic,staged,staged_seg128,pipe_seg512 \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep.jsonl 2> gpurun_out/${T}_sweep.err || exit 4
SWEEP_ROUNDS=1 SWEEP_ONLY=automatic timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep_pow2.jsonl 2> gpurun_out/${T}_sweep_pow2.err || exit 5
