#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T=$1
DIAG_BATCHES=0 RSG_TIMING=1 timeout -k 10 100 python -u tools/diag_cfg3.py 1 > gpurun_out/${T}_diag.log 2>&1
echo "rc=$?" >> gpurun_out/${T}_diag.log
grep -v "v.plan\|v.kernel\|v.resolve" gpurun_out/${T}_diag.log > gpurun_out/${T}_diag_short.log
rm -f gpurun_out/${T}_diag.log
