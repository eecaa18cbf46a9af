set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06w
mkdir -p gpurun_out
SWEEP_BLENS=1000,1224,1448,2000,2289,3504,4000,6000,8000,9000,12000,16000,20000,24577,32769,65537 SWEEP_ONLY=automatic,lines,staged,pipe_seg512 timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/${T}_blens.jsonl 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 7; }
python - <<'PY'
import json
for l in open('gpurun_out/r06w_blens.jsonl'):
    d=json.loads(l); v=d['variants']
    print(d['block_len'], {k: v[k]['kernel_ms'] for k in v})
PY
timeout -k 10 300 python tools/blocklen_sweep.py --unaligned > gpurun_out/${T}_unal.jsonl 2>> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 8; }
cut -c1-400 gpurun_out/${T}_unal.jsonl
