set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05w
for r in 1 2; do
  for c in 24 32 40; do
    RSG_CONFIRM_CUS=$c timeout -k 10 120 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_c${c}_$r.json 2> ${P}_cfg3_c${c}_$r.err || exit 4
  done
done
