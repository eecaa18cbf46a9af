set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05s
T="--timeout 120 --timeout-method thread"
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q $T > ${P}_pytest.log 2>&1 || { tail -30 ${P}_pytest.log; exit 2; }
for r in 1 2 3; do
  for m in 1 0; do
    RSG_START_SERIAL=$m timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_s${m}_$r.json 2> ${P}_cfg3_s${m}_$r.err || exit 4
  done
done
RSG_TIMING=1 timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path --steps 3 > ${P}_cfg3_timing.json 2> ${P}_cfg3_timing.err || exit 5
