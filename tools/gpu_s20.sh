set -o pipefail
mkdir -p gpurun_out
for r in 1 2; do
  echo "plain $r"; timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s20_plain_r$r.json 2>/dev/null || exit 1
  echo "hwq8 $r"; GPU_MAX_HW_QUEUES=8 timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s20_hwq8_r$r.json 2>/dev/null || exit 1
  echo "traced $r"; timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_s20_r$r -o trace -- python3 bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s20_traced_r$r.log 2>&1 || exit 1
done
echo done
