set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06l
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_filesums.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
timeout -k 10 300 python bench.py --workload filesums --no-cpu > gpurun_out/${T}_filesums.json 2> gpurun_out/${T}_filesums.err || { tail -20 gpurun_out/${T}_filesums.err; exit 5; }
python -c "import json;d=json.load(open('gpurun_out/${T}_filesums.json'));print(d['modes'])"
PASSES="FETCH_SIZE;WRITE_SIZE" timeout -k 10 400 bash tools/profile_kernel.sh ${T}_filesums file_sums --workload filesums --no-cpu --steps 10 --warmup 2 || exit 6
SWEEP_SQRT=1 SWEEP_ONLY=automatic RSG_LIB_PATH=rsync_amd/ab/librsg_diag_a16.so timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sqrt_a16.jsonl 2> gpurun_out/${T}_sqrt_a16.err || { tail -20 gpurun_out/${T}_sqrt_a16.err; exit 7; }
cut -c1-200 gpurun_out/${T}_sqrt_a16.jsonl
