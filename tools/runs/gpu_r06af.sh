set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06af
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py tests/test_gpu_sender_fd.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -k cfg3 -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_t2.log 2>&1 || { tail -40 gpurun_out/${T}_t2.log; exit 1; }
tail -1 gpurun_out/${T}_t2.log
for r in 1 2 3; do
for lib in rsync_amd/librsg.so rsync_amd/ab/librsg_rollprev.so; do
n=$(basename $lib .so)
RSG_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu > gpurun_out/${T}_cfg3_${n}_$r.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg3_${n}_$r.json'));r=d['roofline'];print('$n', d['value'], 'roll', r['kernel_ms'], 'confirm', r['confirm_ms_per_batch'], 'cand', r['candidates_per_launch'])"
done
done
