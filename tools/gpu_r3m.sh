#!/bin/bash
# Sender parity, then the cfg3 line twice (same box).
set -o pipefail
mkdir -p gpurun_out
T=$1
timeout -k 10 500 python -u -m pytest tests/test_gpu_match.py -x -v --timeout 120 --timeout-method thread \
  > gpurun_out/${T}_match.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 240 python -u bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/${T}_cfg3_$k.json 2> gpurun_out/${T}_cfg3_$k.err || exit 2
done
RSG_TIMING=1 DIAG_BATCHES=1 timeout -k 10 100 python -u tools/diag_cfg3.py 3 2>&1 | grep -v "v.plan\|v.kernel\|v.resolve" > gpurun_out/${T}_timing.log
