set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06v
mkdir -p gpurun_out
for r in 1 2; do
SWEEP_SQRT=2,3,17,33 SWEEP_ONLY=lines timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_def_$r.jsonl 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 7; }
RSG_LINES_NT=1 SWEEP_SQRT=2,3,17,33 SWEEP_ONLY=lines timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_nt_$r.jsonl 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 7; }
done
python - <<'PY'
import json
for r in (1,2):
    a=[json.loads(l) for l in open(f'gpurun_out/r06v_def_{r}.jsonl')]
    b=[json.loads(l) for l in open(f'gpurun_out/r06v_nt_{r}.jsonl')]
    for x,y in zip(a,b): print(r, x['block_len'], 'default', x['variants']['lines']['kernel_ms'], 'nt', y['variants']['lines']['kernel_ms'])
PY
