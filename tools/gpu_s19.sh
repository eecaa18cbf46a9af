set -o pipefail
mkdir -p gpurun_out
T="--timeout 200 --timeout-method thread"
echo "match tests"; timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s19_pytest.log 2>&1 || exit 1
for r in 1 2; do
  for b in 0 1; do
    echo "cfg3 blocking=$b run $r"; RSG_BLOCKING_SYNC=$b timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s19_cfg3_b${b}_r$r.json 2>/dev/null || exit 1
  done
done
export PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SALU;FETCH_SIZE"
bash tools/profile_kernel.sh r03m_roll roll_kernel --workload cfg3 --steps 2 --warmup 1 --cfg3-files 4 --no-cpu || exit 1
echo done
