#!/bin/bash
# Packed roll filter bits A/B (RSG_ROLL_BITS 2 / 3), interleaved, same box; parity with 3 bits first.
set -o pipefail
mkdir -p gpurun_out
T=$1
RSG_ROLL_BITS=3 timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_match3.log 2>&1 || exit 1
for k in 1 2; do for NB in 2 3; do
  RSG_ROLL_BITS=$NB timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/${T}_cfg3_b${NB}_$k.json 2> gpurun_out/${T}_b${NB}_$k.err || exit 2
done; done
