set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05o
T="--timeout 120 --timeout-method thread"
RSG_CONFIRM_SPEC=0 timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_sender_fd.py -m gpu -x -q $T > ${P}_pytest_raw.log 2>&1 || { tail -30 ${P}_pytest_raw.log; exit 2; }
RSG_CONFIRM_SPEC=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q $T -k "cfg3" > ${P}_pytest_raw_large.log 2>&1 || { tail -30 ${P}_pytest_raw_large.log; exit 3; }
for r in 1 2 3; do
  RSG_CONFIRM_SPEC=1 timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_spec$r.json 2> ${P}_cfg3_spec$r.err || exit 4
  RSG_CONFIRM_SPEC=0 timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_raw$r.json 2> ${P}_cfg3_raw$r.err || exit 5
done
BENCH_DELIVERY_DIAG=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-path > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 6
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-host-path > ${P}_cfg4.json 2> ${P}_cfg4.err || exit 7
