set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05q
export TMPDIR=/tmp
T="--timeout 120 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_sender_fd.py -m gpu -x -q $T > ${P}_pytest.log 2>&1 || { tail -30 ${P}_pytest.log; exit 2; }
RSG_CONFIRM_SPEC=0 timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_match.py -m gpu -x -q $T > ${P}_pytest_raw.log 2>&1 || { tail -30 ${P}_pytest_raw.log; exit 3; }
for r in 1 2; do
  for m in 1 0; do for sp in 0 1; do
    RSG_CU_MASK=$m RSG_CONFIRM_SPEC=$sp timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_m${m}s${sp}_$r.json 2> ${P}_cfg3_m${m}s${sp}_$r.err || exit 4
  done; done
done
RSG_CONFIRM_SPEC=0 timeout -k 10 -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d ${P}_trace -o trace -- python3 bench.py --workload cfg3 --steps 3 --warmup 1 --no-cpu --no-host-path > ${P}_cfg3_trace.log 2>&1 || exit 5
BENCH_DELIVERY_DIAG=2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-path > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 6
