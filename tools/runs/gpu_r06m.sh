set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06m
mkdir -p gpurun_out
export TMPDIR=/tmp
for m in 1 2 3 9; do
  for P in FETCH_SIZE WRITE_SIZE; do
    SWEEP_SQRT=$m SWEEP_ONLY=automatic timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex block_sums --output-format csv -d gpurun_out/prof_${T}_m$m/pmc_$P -o pmc -- python3 tools/blocklen_sweep.py > gpurun_out/${T}_m${m}_$P.log 2>&1 || { echo "pmc $m $P failed"; exit 3; }
  done
  echo "done $m"
done
