#!/bin/bash
# PMC passes (separate from any trace) for one block-sum kernel variant.
# Usage: tools/pmc_variant.sh <variant> <tag>
set -o pipefail
V=$1; TAG=$2
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
export RSG_BLOCKSUMS_KERNEL=$V
for P in "FETCH_SIZE" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $P --output-format csv -d $OUT/$N -o pmc -- python3 bench.py --steps 20 --warmup 100 --no-cpu --no-host-path > $OUT/$N.log 2>&1 || exit 1
done
