set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  for b in 0 1; do
    echo "cfg3 blocking=$b run $r"; RSG_BLOCKING_SYNC=$b timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s18_cfg3_b${b}_r$r.json 2>/dev/null || exit 1
  done
done
echo "cfg3 overlap0"; RSG_SEARCH_OVERLAP=0 timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s18_cfg3_ov0.json 2>/dev/null || exit 1
echo "trace plain-ish"; timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_r03l_cfg3 -o trace -- python3 bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/prof_r03l_cfg3.log 2>&1 || exit 1
echo done
