set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_blocksums.py -k "persistent_waves_many_groups or variants_device_aligned_arena or (kernel_variants_match and (13 or 14 or 15))" > gpurun_out/r05at_tests.log 2>&1 || exit 3
SWEEP_SHAPES=1,4,2 SWEEP_ROUNDS=2 SWEEP_ONLY=automatic,staged_seg128,pipe_seg128,pipe_seg128_imm,pipe_seg512,diag_pipe_seg128_memory_only \
  timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/r05at_sweep.jsonl 2> gpurun_out/r05at_sweep.err || exit 4
SWEEP_BLENS=1000,1448,2000,4000,6000 SWEEP_ONLY=automatic,staged,pipe_seg128,pipe_seg128_imm,pipe_seg512 \
  timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/r05at_sweep2.jsonl 2> gpurun_out/r05at_sweep2.err || exit 5
