set -o pipefail
cd $GRAFT_REPO_ROOT
P=gpurun_out/r05ah
s=$(date +%s)
timeout -k 10 600 python bench.py > ${P}_default.json 2> ${P}_default.err || exit 2
echo "default bench wall $(( $(date +%s) - s )) s"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit 3
