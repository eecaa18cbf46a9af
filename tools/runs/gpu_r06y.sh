set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06y
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_blocksums.py tests/test_gpu_match.py tests/test_abi.py tests/test_c_abi.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_large.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_t2.log 2>&1 || { tail -40 gpurun_out/${T}_t2.log; exit 1; }
tail -1 gpurun_out/${T}_t2.log
SWEEP_SQRT=1 SWEEP_ONLY=automatic timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sqrt.jsonl 2> gpurun_out/${T}_sqrt.err || { tail -20 gpurun_out/${T}_sqrt.err; exit 7; }
cut -c1-220 gpurun_out/${T}_sqrt.jsonl
for r in 1 2; do
timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu > gpurun_out/${T}_cfg3_$r.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg3_$r.json'));r=d['roofline'];print(d['value'], 'roll', r['kernel_ms'], 'confirm', r['confirm_ms_per_batch'], d['call_ms'])"
done
