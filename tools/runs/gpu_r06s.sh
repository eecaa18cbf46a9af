set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06s
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blocksums.py tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 200 python tools/confirm_probe.py 32768 64 2368 23515 > gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 3; }
cat gpurun_out/${T}_probe.jsonl
for r in 1 2; do
timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu > gpurun_out/${T}_cfg3_$r.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg3_$r.json'));r=d['roofline'];print(d['value'], 'roll', r['kernel_ms'], 'confirm', r['confirm_ms_per_batch'], d['call_ms'])"
done
