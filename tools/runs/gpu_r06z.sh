set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06z
mkdir -p gpurun_out
for r in 1 2; do
timeout -k 10 300 python bench.py --workload filesums --no-cpu > gpurun_out/${T}_fs_$r.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 5; }
RSG_LIB_PATH=rsync_amd/ab/librsg_diag_fsmem.so timeout -k 10 300 python bench.py --workload filesums --no-cpu > gpurun_out/${T}_fsmem_$r.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 5; }
python -c "
import json
a=json.load(open('gpurun_out/${T}_fs_$r.json'))['modes']; b=json.load(open('gpurun_out/${T}_fsmem_$r.json'))['modes']
print('product', a['seeded']['kernel_ms'], a['plain']['kernel_ms'], 'memory-only', b['seeded']['kernel_ms'], b['plain']['kernel_ms'])"
done
