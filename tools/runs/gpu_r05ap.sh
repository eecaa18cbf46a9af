set -o pipefail
cd $GRAFT_REPO_ROOT
T=r05ap
bash tools/gpu_run.sh $T tests smoke bench || exit 1
SWEEP_ROUNDS=2 SWEEP_ONLY=automatic,staged_seg128,staged_seg128_persist,pipe_seg128,pipe_seg512,pipe,diag_staged_seg128_memory_only,diag_pipe_seg128_memory_only \
  timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep.jsonl 2> gpurun_out/${T}_sweep.err || exit 4
