#!/bin/bash
# cfg3 A/B: the confirmation kernel (RSG_BLOCKSUMS_KERNEL: -1 auto = unaligned
# staged, 3 = deep per-lane prefetch) x the CUs the roll leaves to it
# (RSG_CONFIRM_CUS, 0 = confirmation queued behind the next roll).
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_blocksums.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || exit 1
for kv in -1 3; do
  for k in 0 16 24 32; do
    RSG_BLOCKSUMS_KERNEL=$kv RSG_CONFIRM_CUS=$k timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/ab_cfg3_v${kv}_k$k.json 2> gpurun_out/ab_cfg3_v${kv}_k$k.err || exit 1
  done
done
