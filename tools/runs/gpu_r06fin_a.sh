# Final evidence pass, part A: the whole GPU suite once, then smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_run.sh r06fin tests smoke || exit 1
tail -3 gpurun_out/r06fin_pytest.log
