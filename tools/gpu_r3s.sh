#!/bin/bash
# The >4 GiB sender test, then the default cfg3 line (CPU baseline, oracle parity on file 0).
set -o pipefail
mkdir -p gpurun_out
T=${1:-s1}
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -k "sender_search_past_4gib or release" -x -v --timeout 240 --timeout-method thread \
  > gpurun_out/${T}_large.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --workload cfg3 > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || exit 2
