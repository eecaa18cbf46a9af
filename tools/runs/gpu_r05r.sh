set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05r
T="--timeout 120 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_sender_fd.py -m gpu -x -q $T > ${P}_pytest.log 2>&1 || { tail -30 ${P}_pytest.log; exit 2; }
for r in 1 2; do
  for c in 24 32 40 48 64; do
    RSG_CONFIRM_CUS=$c timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_c${c}_$r.json 2> ${P}_cfg3_c${c}_$r.err || exit 4
  done
done
BENCH_DELIVERY_DIAG=2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu --no-host-path > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 6
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu --no-host-path > ${P}_cfg4.json 2> ${P}_cfg4.err || exit 7
