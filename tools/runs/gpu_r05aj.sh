set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05aj
T="--timeout 150 --timeout-method thread"
RSG_UNAL_SEG=128 timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_blocksums.py -m gpu -x -q $T -k "not full" > ${P}_pytest.log 2>&1 || { tail -40 ${P}_pytest.log; exit 2; }
for r in 1 2 3; do
  for m in 128 256; do
    RSG_UNAL_SEG=$m timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_s${m}_$r.json 2> ${P}_cfg3_s${m}_$r.err || exit 4
  done
done
