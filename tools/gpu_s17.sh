set -o pipefail
mkdir -p gpurun_out
T="--timeout 200 --timeout-method thread"
echo "gpu tests"; timeout -k 10 900 python -u -m pytest tests -x -q -m gpu $T > gpurun_out/s17_pytest.log 2>&1 || exit 1
for r in 1 2 3; do
  echo "cfg3 run $r"; timeout -k 10 120 python bench.py --workload cfg3 --steps 5 --no-cpu > gpurun_out/s17_cfg3_r$r.json 2>/dev/null || exit 1
done
echo "cfg3 steps2"; timeout -k 10 120 python bench.py --workload cfg3 --steps 2 --warmup 1 --no-cpu > gpurun_out/s17_cfg3_s2.json 2>/dev/null || exit 1
echo "cfg3 full line"; timeout -k 10 200 python bench.py --workload cfg3 --steps 5 --cpu-seconds 5 > gpurun_out/s17_cfg3_full.json 2>/dev/null || exit 1
echo "cfg2"; timeout -k 10 300 python bench.py > gpurun_out/s17_cfg2.json 2>gpurun_out/s17_cfg2.err || exit 1
echo done
