# Evidence on the round's last code state: the whole GPU suite once, smoke, the default bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r06end tests smoke bench || exit 1
tail -3 gpurun_out/r06end_pytest.log
python -c "import json;d=json.load(open('gpurun_out/r06end_cfg2.json'));print('cfg2', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'] if 'kernel_ms' in d['roofline'] else '')"
