set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blocksums.py -k "persistent_waves_many_groups or variants_device_aligned_arena or (kernel_variants_match and (13 or 14 or 15))" > gpurun_out/r05am_tests.log 2>&1 || exit 3
SWEEP_SHAPES=2,1,4,0 SWEEP_ROUNDS=2 SWEEP_ONLY=automatic,staged_seg128,staged_seg128_persist,staged_persist,staged,pipe_seg128,pipe_seg512,pipe,diag_staged_seg128_memory_only,diag_staged_seg128_persist_memory_only,diag_pipe_seg128_memory_only,diag_pipe_seg512_memory_only,diag_pipe_memory_only,diag_staged_persist_memory_only,diag_staged_seg512_persist_memory_only \
  timeout -k 10 400 python tools/blocklen_sweep.py > gpurun_out/r05am_sweep.jsonl 2> gpurun_out/r05am_sweep.err
