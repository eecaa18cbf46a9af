set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06ai
mkdir -p gpurun_out
SWEEP_SQRT=1 SWEEP_ROUNDS=3 SWEEP_ONLY=automatic timeout -k 10 400 python tools/blocklen_sweep.py > gpurun_out/${T}_sqrt.jsonl 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 7; }
python - <<'PY'
import json
for l in open('gpurun_out/r06ai_sqrt.jsonl'):
    d=json.loads(l); v=d['variants']['automatic']
    print(d['block_len'], v.get('rounds_ms'), v['hbm_frac_8tbs'])
PY
