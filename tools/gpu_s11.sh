set -o pipefail
mkdir -p gpurun_out
T="--timeout 200 --timeout-method thread"
echo "match tests default"; timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s11_pytest_default.log 2>&1 || exit 1
echo "match tests sel+ring 512"; RSG_FILTER_SEL=1 RSG_ROLL_RING=1 RSG_ROLL_LANES=512 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s11_pytest_512.log 2>&1 || exit 1
echo "match tests sel+ring 1024"; RSG_FILTER_SEL=1 RSG_ROLL_RING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s11_pytest_1024.log 2>&1 || exit 1
echo "blocksums tests"; timeout -k 10 600 python -u -m pytest tests/test_gpu_blocksums.py tests/test_gpu_large.py -x -q -m gpu $T > gpurun_out/s11_pytest_bs.log 2>&1 || exit 1
for r in 1 2; do
  for v in 0_0_1024 1_0_1024 1_1_1024 1_1_512 1_0_512; do
    IFS=_ read e g l <<< "$v"
    echo "cfg3 sel=$e ring=$g lanes=$l round $r"
    RSG_FILTER_SEL=$e RSG_ROLL_RING=$g RSG_ROLL_LANES=$l timeout -k 10 240 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s11_cfg3_${v}_r${r}.json 2>gpurun_out/s11_cfg3_${v}_r${r}.err || exit 1
  done
done
echo cfg2; timeout -k 10 200 python bench.py --no-cpu --no-host-path --no-delivery > gpurun_out/s11_cfg2.json 2>/dev/null || exit 1
export PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SALU"
RSG_FILTER_SEL=1 RSG_ROLL_RING=1 RSG_ROLL_LANES=512 bash tools/profile_kernel.sh r03g_roll_512 roll_kernel --workload cfg3 --steps 2 --warmup 1 --cfg3-files 4 --no-cpu || exit 1
RSG_FILTER_SEL=1 RSG_ROLL_RING=1 bash tools/profile_kernel.sh r03g_roll_1024 roll_kernel --workload cfg3 --steps 2 --warmup 1 --cfg3-files 4 --no-cpu || exit 1
echo done
