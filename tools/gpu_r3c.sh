#!/bin/bash
# cfg3 line at several RSG_CONFIRM_CUS values (same box).
set -o pipefail
mkdir -p gpurun_out
T=$1; shift
for C in "$@"; do
  RSG_CONFIRM_CUS=$C timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu \
    > gpurun_out/${T}_cfg3_c$C.json 2> gpurun_out/${T}_cfg3_c$C.err || exit 2
done
