#!/bin/bash
# Packed roll group size A/B (RSG_ROLL_G 4 / 8 / 2), parity for each, interleaved cfg3 lines.
set -o pipefail
mkdir -p gpurun_out
T=$1
for G in 8 2; do
  RSG_ROLL_G=$G timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${T}_match_g$G.log 2>&1 || exit 1
done
for k in 1 2; do for G in 4 8 2; do
  RSG_ROLL_G=$G timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/${T}_cfg3_g${G}_$k.json 2> gpurun_out/${T}_g${G}_$k.err || exit 2
done; done
