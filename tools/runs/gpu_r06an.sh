set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# whole-file MD4: LDS-DMA copies (0, product) vs register-staged copies, K segments in flight (A/B build, RSG_FS_REGS)
i=0
for k in 0 2 3 4 0; do
  i=$((i+1)); f=gpurun_out/r06an_fs_${i}_k$k
  RSG_FS_REGS=$k timeout -k 10 240 python -u bench.py --workload filesums --steps 20 --cpu-seconds 1 > $f.json 2> $f.err || exit 1
  python -c "import json;d=json.loads(open('$f.json').read().strip().splitlines()[-1]);print('$k', d['modes']['seeded']['kernel_ms'], d['modes']['plain']['kernel_ms'], d['value'], d['spot_parity'])"
done
