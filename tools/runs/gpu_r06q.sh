set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06q
mkdir -p gpurun_out
for r in 1 2; do
for o in confirm_cus=32 confirm_cus=24 confirm_cus=16 confirm_cus=40 spec=1; do
  timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu --search-option $o > gpurun_out/${T}_$o.$r.json 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 6; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_$o.$r.json'));r=d['roofline'];print('$o', d['value'], 'roll', r['kernel_ms'], 'confirm', r['confirm_ms_per_batch'], 'windows', r['windows_confirmed_per_launch'])"
done
done
