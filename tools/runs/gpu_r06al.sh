set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# whole-file MD4 lane order A/B: length-bucket width 2^shift (10 = product)
i=0
for sh in 10 13 40 8 16 10; do
  i=$((i+1)); f=gpurun_out/r06al_fs_${i}_$sh
  timeout -k 10 240 python -u bench.py --workload filesums --steps 20 --cpu-seconds 1 --search-option fs_key_shift=$sh \
    > $f.json 2> $f.err || exit 1
  python -c "import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);print('$sh', d['modes']['seeded']['kernel_ms'], d['modes']['plain']['kernel_ms'], d['value'], d['spot_parity'])"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_filesums.py > gpurun_out/r06al_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/r06al_pytest.log; exit $rc
