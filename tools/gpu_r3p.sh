#!/bin/bash
# Round 3, packed roll: GPU parity of the sender search, then the cfg3 line
# with each roll variant given (RSG_ROLL_PACKED values) on the same box.
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_match.log 2>&1 || exit 1
for V in "$@"; do
  RSG_ROLL_PACKED=$V timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu \
    > gpurun_out/${T}_cfg3_v$V.json 2> gpurun_out/${T}_cfg3_v$V.err || exit 2
done
