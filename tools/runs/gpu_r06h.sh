set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06h
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_filesums.py -m gpu -x -q --timeout 100 --timeout-method thread > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
timeout -k 10 300 python bench.py --workload filesums --no-cpu > gpurun_out/${T}_filesums.json 2> gpurun_out/${T}_filesums.err || { tail -20 gpurun_out/${T}_filesums.err; exit 5; }
cat gpurun_out/${T}_filesums.json
PASSES="FETCH_SIZE;WRITE_SIZE;SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE" timeout -k 10 600 bash tools/profile_kernel.sh ${T}_filesums file_sums --workload filesums --no-cpu --steps 10 --warmup 2 || exit 6
