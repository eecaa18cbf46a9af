set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06aj
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sender_small.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
for r in 1 2 3; do
for lib in rsync_amd/librsg.so rsync_amd/ab/librsg_smallprev.so; do
n=$(basename $lib .so)
RSG_LIB_PATH=$lib timeout -k 10 400 python bench.py --workload cfg4-sender --steps 5 --no-cpu > gpurun_out/${T}_${n}_$r.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/${T}_${n}_$r.json'));print('$n', d['value'], d['call_ms'], d['roofline']['launches_per_call'])"
done
done
