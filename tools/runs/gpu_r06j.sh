set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06j
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_blocksums.py -k "sqrt or automatic_rule" -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/${T}_tb.log 2>&1 || { tail -40 gpurun_out/${T}_tb.log; exit 1; }
for ch in 421 431 430 230 240 220 402; do
  RSG_FS_CH=$ch timeout -k 10 200 python -u -m pytest tests/test_gpu_filesums.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/${T}_t_$ch.log 2>&1 || { tail -40 gpurun_out/${T}_t_$ch.log; exit 1; }
  RSG_FS_CH=$ch timeout -k 10 300 python bench.py --workload filesums --no-cpu > gpurun_out/${T}_filesums_$ch.json 2> gpurun_out/${T}_filesums_$ch.err || { tail -20 gpurun_out/${T}_filesums_$ch.err; exit 5; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_filesums_$ch.json'));print($ch, d['modes'])"
done
