#!/bin/bash
# Kernel trace of the cfg3 bench with the lane-slot roll (RSG_ROLL_PACKED=2).
set -o pipefail
T=${1:-t1}
export RSG_ROLL_PACKED=2
OUT=gpurun_out/prof_$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py --workload cfg3 --cfg3-files 4 --steps 2 --no-cpu > $OUT/trace.log 2>&1 || exit 1
