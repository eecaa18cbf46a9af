#!/bin/bash
# rocprofv3 evidence for the sender (cfg3): kernel trace + stats, then
# separate PMC passes (never combined with trace domains).
# Usage: tools/profile_cfg3.sh <tag>
set -o pipefail
TAG=${1:-r02}
OUT=gpurun_out/prof_cfg3_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
ARGS="--workload cfg3 --cfg3-files 2 --steps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
for P in "FETCH_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "roll_kernel" --output-format csv -d $OUT/pmc_$N -o pmc -- python3 bench.py $ARGS > $OUT/pmc_$N.log 2>&1 || echo "pmc pass $P failed rc=$?" >> $OUT/errors.txt
done
exit 0
