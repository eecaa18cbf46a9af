set -o pipefail
mkdir -p gpurun_out
echo "match tests pipe+k3"; RSG_ROLL_PIPE=1 RSG_FILTER_K3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/s10_pytest.log 2>&1 || exit 1
for r in 1 2; do
  for v in 00 10 01 11; do
    p=${v:0:1}; k=${v:1:1}
    echo "cfg3 pipe=$p k3=$k round $r"
    RSG_ROLL_PIPE=$p RSG_FILTER_K3=$k timeout -k 10 240 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s10_cfg3_${v}_r${r}.json 2>gpurun_out/s10_cfg3_${v}_r${r}.err || exit 1
  done
done
export PASSES="FETCH_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SALU"
bash tools/profile_kernel.sh r03f_roll roll_kernel --workload cfg3 --steps 2 --warmup 1 --cfg3-files 4 --no-cpu || exit 1
for r in 1 2 3; do
  for L in head cur; do
    if [ $L = head ]; then export RSG_LIB_PATH=$PWD/rsync_amd/ab/librsg_head.so; else unset RSG_LIB_PATH; fi
    echo "order A/B $L round $r"
    timeout -k 10 200 python bench.py --steps 100 --windows 3 --no-cpu --no-host-path --no-delivery > gpurun_out/s10_cfg2_${L}_r${r}.json 2>/dev/null || exit 1
    timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --windows 3 --no-cpu --no-delivery > gpurun_out/s10_cfg4_${L}_r${r}.json 2>/dev/null || exit 1
  done
done
unset RSG_LIB_PATH
echo done
