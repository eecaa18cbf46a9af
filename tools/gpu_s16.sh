set -o pipefail
mkdir -p gpurun_out
T="--timeout 200 --timeout-method thread"
echo "match tests default"; timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s16_pytest_default.log 2>&1 || exit 1
echo "match tests all=0"; RSG_CONFIRM_ALL=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s16_pytest_call0.log 2>&1 || exit 1
echo "match tests overlap=0"; RSG_SEARCH_OVERLAP=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s16_pytest_ov0.log 2>&1 || exit 1
echo "match tests sel=0"; RSG_FILTER_SEL=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_match.py -x -q -m gpu $T > gpurun_out/s16_pytest_sel0.log 2>&1 || exit 1
for r in 1 2; do
  for v in 1_1 1_0 0_1; do
    IFS=_ read e a <<< "$v"
    echo "cfg3 sel=$e all=$a round $r"
    RSG_FILTER_SEL=$e RSG_CONFIRM_ALL=$a timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s16_cfg3_${v}_r${r}.json 2>gpurun_out/s16_cfg3_${v}_r${r}.err || exit 1
  done
done
echo "cus"; for c in 24 40; do RSG_CONFIRM_CUS=$c timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s16_cfg3_cus$c.json 2>/dev/null || exit 1; done
echo "trace"; timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r03k_cfg3 -o trace -- python3 bench.py --workload cfg3 --steps 2 --warmup 1 --cfg3-files 10 --no-cpu > gpurun_out/prof_r03k_cfg3.log 2>&1 || exit 1
echo done
