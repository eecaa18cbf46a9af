#!/bin/bash
# cfg3 line for each roll variant given (RSG_ROLL_PACKED values), same box.
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
for V in "$@"; do
  RSG_ROLL_PACKED=$V timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu \
    > gpurun_out/${T}_cfg3_v$V.json 2> gpurun_out/${T}_cfg3_v$V.err || exit 2
done
