#!/bin/bash
# Packed roll, edge tiles inside (RSG_ROLL_EDGE=1, default) vs a separate
# roll_kernel launch (0): sender parity for both, then interleaved cfg3 lines.
set -o pipefail
mkdir -p gpurun_out
T=$1
for E in 1 0; do
  RSG_ROLL_EDGE=$E timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_match_e$E.log 2>&1 || exit 1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "sender_search_past_4gib or release" -x -q --timeout 240 --timeout-method thread \
  > gpurun_out/${T}_large.log 2>&1 || exit 1
for k in 1 2 3; do for E in 1 0; do
  RSG_ROLL_EDGE=$E timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/${T}_cfg3_e${E}_$k.json 2> gpurun_out/${T}_e${E}_$k.err || exit 2
done; done
