set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06t
mkdir -p gpurun_out
RSG_ROLL_TPB=512 timeout -k 10 400 python -u -m pytest tests/test_gpu_match.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
RSG_ROLL_TPB=512 timeout -k 10 400 python -u -m pytest tests/test_gpu_large.py -k cfg3 -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_t2.log 2>&1 || { tail -40 gpurun_out/${T}_t2.log; exit 1; }
tail -1 gpurun_out/${T}_t2.log
for r in 1 2; do
for tpb in 1024 512; do
RSG_ROLL_TPB=$tpb timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu > gpurun_out/${T}_cfg3_${tpb}_$r.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg3_${tpb}_$r.json'));r=d['roofline'];print($tpb, d['value'], 'roll', r['kernel_ms'], 'confirm', r['confirm_ms_per_batch'], 'cand', r['candidates_per_launch'])"
done
done
