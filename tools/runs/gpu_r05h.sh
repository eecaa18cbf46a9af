# round-5 GPU step h: coalesced nontemporal record stores in park (product)
# and staged kernels -- parity, then A/B against rsync_amd/ab/librsg_base.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/r05h
BASE=$PWD/rsync_amd/ab/librsg_base.so
T="--timeout 120 --timeout-method thread"
timeout -k 10 500 python -u -m pytest -x -v $T tests/test_gpu_blocksums.py tests/test_gpu_large.py tests/test_gpu_match.py tests/test_gpu_generate.py tests/test_dist.py -m gpu > ${P}_pytest.log 2>&1 || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > ${P}_smoke.log 2>&1 || exit 2
timeout -k 10 200 python bench.py > ${P}_cfg2.json 2> ${P}_cfg2.err || exit 3
RSG_LIB_PATH=$BASE timeout -k 10 200 python bench.py --no-cpu --no-host-path --no-delivery > ${P}_cfg2_base.json 2> ${P}_cfg2_base.err || exit 4
timeout -k 10 200 python bench.py --no-cpu --no-host-path --no-delivery > ${P}_cfg2_new2.json 2> ${P}_cfg2_new2.err || exit 5
SWEEP_SHAPES=1,2,4,0,8 timeout -k 10 300 python tools/blocklen_sweep.py > ${P}_sweep_new.jsonl 2> ${P}_sweep_new.err || exit 6
SWEEP_SHAPES=1,2,4,0,8 RSG_LIB_PATH=$BASE timeout -k 10 300 python tools/blocklen_sweep.py > ${P}_sweep_base.jsonl 2> ${P}_sweep_base.err || exit 7
timeout -k 10 200 python bench.py --workload cfg4 --steps 50 > ${P}_cfg4.json 2> ${P}_cfg4.err || exit 8
RSG_LIB_PATH=$BASE timeout -k 10 200 python bench.py --workload cfg4 --steps 50 --no-cpu > ${P}_cfg4_base.json 2> ${P}_cfg4_base.err || exit 9
timeout -k 10 200 python bench.py --workload cfg5 --steps 20 --no-cpu > ${P}_cfg5.json 2> ${P}_cfg5.err || exit 10
RSG_LIB_PATH=$BASE timeout -k 10 200 python bench.py --workload cfg5 --steps 20 --no-cpu > ${P}_cfg5_base.json 2> ${P}_cfg5_base.err || exit 11
