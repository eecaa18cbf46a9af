# round-5 GPU step: parity of the changed paths, then the A/B measurements
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
[ -n "$SKIP_TESTS" ] || timeout -k 10 500 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_match.py tests/test_gpu_sender_fd.py tests/test_shard_plan.py "tests/test_gpu_large.py::test_cfg3_real_size_vs_oracle" > gpurun_out/r05d_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > gpurun_out/r05d_ab.json 2> gpurun_out/r05d_ab.err || exit 2
timeout -k 10 300 python bench.py --workload cfg3 --no-cpu > gpurun_out/r05d_cfg3_spec1.json 2> gpurun_out/r05d_cfg3_spec1.err || exit 3
RSG_CONFIRM_SPEC=0 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/r05d_cfg3_nospec1.json 2> gpurun_out/r05d_cfg3_nospec1.err || exit 4
timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/r05d_cfg3_spec2.json 2> gpurun_out/r05d_cfg3_spec2.err || exit 5
RSG_CONFIRM_SPEC=0 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/r05d_cfg3_nospec2.json 2> gpurun_out/r05d_cfg3_nospec2.err || exit 6
SWEEP_SHAPES=2,5,6,7,8 timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/r05d_sweep.jsonl 2> gpurun_out/r05d_sweep.err || exit 7
