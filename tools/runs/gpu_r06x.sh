set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06x
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_blocksums.py -m gpu -x -q --timeout 200 --timeout-method thread -k "7 or line or sqrt" > gpurun_out/${T}_t1.log 2>&1 || { tail -40 gpurun_out/${T}_t1.log; exit 1; }
tail -1 gpurun_out/${T}_t1.log
SWEEP_BLENS=1000,1224,1448,2000,2289,3504,4000,6000,8000,9000,12000,16000,20000,24577,32769,65537,1773,4222,5882 SWEEP_ONLY=automatic,lines timeout -k 10 500 python tools/blocklen_sweep.py > gpurun_out/${T}_blens.jsonl 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 7; }
python - <<'PY'
import json
for l in open('gpurun_out/r06x_blens.jsonl'):
    d=json.loads(l); v=d['variants']
    print(d['block_len'], {k: v[k]['kernel_ms'] for k in v})
PY
