set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r06ak cfg4s || exit 1
python -c "import json;d=json.load(open('gpurun_out/r06ak_cfg4s.json'));print(d['value'], d['call_ms'], d.get('oracle_parity'), d['cpu_baseline']['value'])"
