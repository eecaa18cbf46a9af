#!/bin/bash
# Round-3 evidence: tools/final_evidence.sh (suite, smoke, every workload,
# cfg2 rocprof), then the cfg3 roll kernel trace + counters.
set -o pipefail
T=${1:-r03r}
bash tools/final_evidence.sh $T || exit 1
PASSES="FETCH_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" \
  timeout -k 10 700 tools/profile_kernel.sh ${T}_cfg3 "roll" --workload cfg3 --cfg3-files 2 --steps 2 --no-cpu || exit 2
