# round-5 GPU step e: roll carry change parity, cfg2 memory diagnostics,
# cfg3 A/B (new library vs rsync_amd/ab/librsg_base.so, speculative
# confirmation on/off), block-length probes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P=gpurun_out/r05e
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_match.py "tests/test_gpu_large.py::test_cfg3_real_size_vs_oracle" "tests/test_gpu_large.py::test_sender_search_past_4gib" > ${P}_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > ${P}_ab.json 2> ${P}_ab.err || exit 2
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu > ${P}_cfg3_new1.json 2> ${P}_cfg3_new1.err || exit 3
RSG_LIB_PATH=$PWD/rsync_amd/ab/librsg_base.so timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_base1.json 2> ${P}_cfg3_base1.err || exit 4
RSG_CONFIRM_SPEC=0 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_nospec1.json 2> ${P}_cfg3_nospec1.err || exit 5
timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_new2.json 2> ${P}_cfg3_new2.err || exit 6
RSG_LIB_PATH=$PWD/rsync_amd/ab/librsg_base.so timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_base2.json 2> ${P}_cfg3_base2.err || exit 7
RSG_CONFIRM_SPEC=0 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_nospec2.json 2> ${P}_cfg3_nospec2.err || exit 8
SWEEP_SHAPES=2,5,6,7,8 timeout -k 10 300 python tools/blocklen_sweep.py > ${P}_sweep.jsonl 2> ${P}_sweep.err || exit 9
RSG_CONFIRM_CUS=24 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_cus24.json 2> ${P}_cfg3_cus24.err || exit 10
RSG_CONFIRM_CUS=16 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > ${P}_cfg3_cus16.json 2> ${P}_cfg3_cus16.err || exit 11
