set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06z2
mkdir -p gpurun_out
for sh in 81 41 42; do
RSG_FS_SHAPE=$sh timeout -k 10 200 python -u -m pytest tests/test_gpu_filesums.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/${T}_t_$sh.log 2>&1 || { tail -30 gpurun_out/${T}_t_$sh.log; exit 1; }
done
for r in 1 2; do
for sh in 81 41 42; do
RSG_FS_SHAPE=$sh timeout -k 10 300 python bench.py --workload filesums --no-cpu > gpurun_out/${T}_fs_${sh}_$r.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 5; }
python -c "
import json
a=json.load(open('gpurun_out/${T}_fs_${sh}_$r.json'))['modes']
print($sh, a['seeded']['kernel_ms'], a['plain']['kernel_ms'])"
done
done
