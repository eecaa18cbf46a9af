set -o pipefail
mkdir -p gpurun_out
T="--timeout 200 --timeout-method thread"
echo "match tests default"; timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s12_pytest_default.log 2>&1 || exit 1
echo "match tests sel+ring"; RSG_FILTER_SEL=1 RSG_ROLL_RING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s12_pytest_selring.log 2>&1 || exit 1
echo "match tests host-batched confirm"; RSG_CONFIRM_ALL=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s12_pytest_call0.log 2>&1 || exit 1
for r in 1 2; do
  for v in 0_0_0 0_0_1 1_0_1 1_1_1; do
    IFS=_ read e g a <<< "$v"
    echo "cfg3 sel=$e ring=$g all=$a round $r"
    RSG_FILTER_SEL=$e RSG_ROLL_RING=$g RSG_CONFIRM_ALL=$a timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s12_cfg3_${v}_r${r}.json 2>gpurun_out/s12_cfg3_${v}_r${r}.err || exit 1
  done
done
echo "timing"; RSG_TIMING=1 timeout -k 10 120 python bench.py --workload cfg3 --steps 1 --warmup 1 --cfg3-files 4 --no-cpu > gpurun_out/s12_timing.json 2>gpurun_out/s12_timing.err || exit 1
echo done
