set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06n
mkdir -p gpurun_out
export TMPDIR=/tmp
for lib in rsync_amd/librsg.so rsync_amd/ab/librsg_diag_aux0.so; do
  SWEEP_SQRT=2,3,17 SWEEP_ROUNDS=2 SWEEP_ONLY=automatic RSG_LIB_PATH=$lib timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_$(basename $lib .so).jsonl 2> gpurun_out/${T}_sw.err || { tail -20 gpurun_out/${T}_sw.err; exit 7; }
  cut -c1-250 gpurun_out/${T}_$(basename $lib .so).jsonl
done
for m in 2 3; do
  SWEEP_SQRT=$m SWEEP_ONLY=automatic RSG_LIB_PATH=rsync_amd/ab/librsg_diag_aux0.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex block_sums --output-format csv -d gpurun_out/prof_${T}_m$m/pmc_FETCH_SIZE -o pmc -- python3 tools/blocklen_sweep.py > gpurun_out/${T}_m${m}.log 2>&1 || { echo "pmc $m failed"; exit 3; }
done
