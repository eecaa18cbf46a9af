set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06ac
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sender_small.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
for r in 1 2; do
for cj in 16384 8192 4096; do
RSG_SMALL_CHUNK=$cj timeout -k 10 400 python bench.py --workload cfg4-sender --steps 5 --no-cpu > gpurun_out/${T}_cfg4s_$cj.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 4; }
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg4s_$cj.json'));print($cj, d['value'], d['call_ms'], d['roofline']['kernel_ms_per_call'], d['roofline']['launches_per_call'])"
done
done
