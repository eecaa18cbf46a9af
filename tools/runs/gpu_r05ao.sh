set -o pipefail
cd $GRAFT_REPO_ROOT
SWEEP_SHAPES=2,1,4 SWEEP_ROUNDS=2 SWEEP_ONLY=automatic,staged_seg128,staged_seg128_persist,pipe_seg128,staged_seg128_uloc,staged_seg128_persist_uloc,diag_staged_seg128_memory_only,diag_staged_seg128_uloc_memory_only,diag_pipe_seg128_memory_only \
  timeout -k 10 400 python tools/blocklen_sweep.py > gpurun_out/r05ao_sweep.jsonl 2> gpurun_out/r05ao_sweep.err
