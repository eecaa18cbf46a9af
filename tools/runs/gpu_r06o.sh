set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06o
mkdir -p gpurun_out
for lib in rsync_amd/librsg.so rsync_amd/ab/librsg_diag_aux0.so; do
  n=$(basename $lib .so)
  SWEEP_BLENS=1000,1448,2000,2289,3504,4000,4222,5882,6000,8000,1773,12000,20000 SWEEP_ONLY=automatic RSG_LIB_PATH=$lib timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_$n.jsonl 2> gpurun_out/${T}_sw.err || { tail -20 gpurun_out/${T}_sw.err; exit 7; }
  RSG_LIB_PATH=$lib timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu > gpurun_out/${T}_cfg3_$n.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_cfg3_$n.json'));print('$n', d['value'], d.get('kernel_times_ms_per_call') or d.get('phases'))"
done
python - <<'PY'
import json
a=[json.loads(l) for l in open('gpurun_out/r06o_librsg.jsonl')]
b=[json.loads(l) for l in open('gpurun_out/r06o_librsg_diag_aux0.jsonl')]
for x,y in zip(a,b): print(x['block_len'], x['variants']['automatic']['kernel_ms'], y['variants']['automatic']['kernel_ms'])
PY
