#!/bin/bash
# Counters of the packed roll variants on cfg3 (RSG_ROLL_PACKED from the env).
set -o pipefail
T=${1:-q1}
PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD" \
  timeout -k 10 600 tools/profile_kernel.sh $T "roll" --workload cfg3 --cfg3-files 2 --steps 2 --no-cpu || exit 1
