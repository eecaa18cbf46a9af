set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# whole-file MD4 lane order A/B: key shift (length buckets) x region shift (0 = off)
i=0
for kr in 10:0 8:0 8:26 8:24 8:22 8:28 8:30 10:0; do
  k=${kr%:*}; r=${kr#*:}
  i=$((i+1)); f=gpurun_out/r06am_fs_${i}_${k}_$r
  timeout -k 10 240 python -u bench.py --workload filesums --steps 20 --cpu-seconds 1 --search-option fs_key_shift=$k \
    --search-option fs_region_shift=$r > $f.json 2> $f.err || exit 1
  python -c "import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);print('$k $r', d['modes']['seeded']['kernel_ms'], d['modes']['plain']['kernel_ms'], d['value'], d['spot_parity'])"
done
