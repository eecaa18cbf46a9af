#!/bin/bash
# Round 3, packed roll: GPU parity of the sender search, then the cfg3 line
# with each roll variant (RSG_ROLL_PACKED = 2 default lane slots, 1 ballots,
# 0 roll_kernel only) on the same box.
set -o pipefail
mkdir -p gpurun_out
T=${1:-p1}
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_match.log 2>&1 || exit 1
for V in 2 1 0 2; do
  RSG_ROLL_PACKED=$V timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu \
    > gpurun_out/${T}_cfg3_v$V.json 2> gpurun_out/${T}_cfg3_v$V.err || exit 2
done
