set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_match.py tests/test_gpu_sender_fd.py > gpurun_out/r05d_pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --ab --no-delivery --no-host-path --no-cpu > gpurun_out/r05d_ab.json 2> gpurun_out/r05d_ab.err || exit 2
for r in 1 2; do
timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/r05d_cfg3_spec$r.json 2> gpurun_out/r05d_cfg3_spec$r.err || exit 3
RSG_CONFIRM_SPEC=0 timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/r05d_cfg3_nospec$r.json 2> gpurun_out/r05d_cfg3_nospec$r.err || exit 4
done
