set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06ag
mkdir -p gpurun_out
for r in 1 2 3; do
for m in nt def; do
if [ $m = def ]; then export RSG_LINES_UNAL_DEFAULT=1; else unset RSG_LINES_UNAL_DEFAULT; fi
timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu > gpurun_out/${T}_cfg3_${m}_$r.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
python -c "import json;d=json.load(open('gpurun_out/${T}_cfg3_${m}_$r.json'));r=d['roofline'];print('$m', d['value'], 'roll', r['kernel_ms'], 'confirm', r['confirm_ms_per_batch'])"
done
done
unset RSG_LINES_UNAL_DEFAULT
