set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05ak
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu --no-host-path > ${P}_default$r.json 2> ${P}_default$r.err || exit 2
done
