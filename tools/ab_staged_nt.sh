mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_blocksums.py -x -q --timeout 120 --timeout-method thread -k "aligned_arena or unaligned_windows" > gpurun_out/s23_pytest.log 2>&1 || exit 1
timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/s23_sweep.jsonl 2> gpurun_out/s23_sweep.err || exit 1
for r in 1 2; do for v in -1 7; do
  RSG_BLOCKSUMS_KERNEL=$v timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/s23_cfg3_r${r}_v$v.json 2>/dev/null || exit 1
done; done
