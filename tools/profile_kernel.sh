#!/bin/bash
# rocprofv3 evidence for one bench workload: a kernel-trace + stats pass, then
# separate PMC passes (never combined with trace domains), each under its own
# time limit; counters only for kernels matching <regex> (keeps the CSVs
# small).  Prints a line per pass so a long run is never silent.
# Usage: tools/profile_kernel.sh <tag> <kernel-regex> <bench args...>
# Summarize afterwards with tools/summarize_profile.py <tag> --kernel <name>.
set -o pipefail
TAG=$1; shift
RX=$1; shift
ARGS="$@"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
echo "[$TAG] trace pass"
# TRACE_ALL=1: trace every kernel (the data fills too: cfg3's trace is then ~50 MB)
if [ -n "$TRACE_ALL" ]; then TRX=""; else TRX="--kernel-include-regex $RX"; fi
timeout -k 10 -s KILL 240 rocprofv3 --kernel-trace --stats $TRX --output-format csv -d $OUT/trace -o trace -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || exit 1
DEFAULT_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE;TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"
# PASSES (optional): counter passes separated by ';'
IFS=';' read -ra PASS_LIST <<< "${PASSES:-$DEFAULT_PASSES}"
for P in "${PASS_LIST[@]}"; do
  N=$(echo $P | tr ' ' '_' | cut -c1-40)
  echo "[$TAG] pmc pass $P"
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_$N -o pmc -- python3 bench.py $ARGS > $OUT/pmc_$N.log 2>&1 || echo "pmc pass $P failed rc=$?" | tee -a $OUT/errors.txt
done
exit 0
