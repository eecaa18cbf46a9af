# Final evidence pass, part B: every workload's bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r06fin bench cfg3 cfg4 cfg5 filesums receive cfg4s sqrt || exit 1
for f in cfg2 cfg3 cfg4 cfg5 filesums receive cfg4s; do python -c "import json;d=json.load(open('gpurun_out/r06fin_$f.json'));print('$f', d['value'], d.get('unit'), (d.get('roofline') or {}).get('frac'))"; done
