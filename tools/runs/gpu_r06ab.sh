set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06ab
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_sender_small.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
RSG_TIMING=1 timeout -k 10 400 python bench.py --workload cfg4-sender --steps 5 --no-cpu > gpurun_out/${T}_cfg4s.json 2> gpurun_out/${T}_cfg4s.err || { tail -20 gpurun_out/${T}_cfg4s.err; exit 4; }
grep "small:" gpurun_out/${T}_cfg4s.err | tail -4
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg4s.json'));print(d['value'], d['call_ms'], d['roofline']['kernel_ms_per_call'], d.get('oracle_parity'))"
