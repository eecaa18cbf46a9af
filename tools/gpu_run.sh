#!/bin/bash
# One gpurun call's worth of GPU work, each step under its own time limit,
# chained so that the first failure (or a hang) ends the call.
#   tools/gpu_run.sh <tag> <step>...   steps: tests | newtests | smoke | sweep | sqrt | variants | ab8 | ab |
#                                             bench | cfg3 | cfg4 | cfg4s | cfg5 | filesums | receive |
#                                             prof_cfg2 | prof_cfg3 | prof_cfg4 | prof_cfg4s | prof_cfg5 | prof_filesums
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
T="--timeout 120 --timeout-method thread"
for S in "$@"; do
  echo "[$TAG] $S $(date +%T)"
  case $S in
    tests) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v $T > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; } ;;
    newtests) timeout -k 10 400 python -u -m pytest tests/test_shard_plan.py tests/test_gpu_sender_fd.py -m gpu -x -v $T > gpurun_out/${TAG}_newtests.log 2>&1 || { tail -30 gpurun_out/${TAG}_newtests.log; exit 1; } ;;
    smoke) timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit 1 ;;
    sweep) SWEEP_SHAPES=${SWEEP_SHAPES:-1,4,2,0} SWEEP_ROUNDS=2 timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${TAG}_sweep.jsonl 2> gpurun_out/${TAG}_sweep.err || exit 1 ;;
    variants) timeout -k 10 300 python -u -m pytest tests/test_gpu_blocksums.py -m gpu -x -q $T -k "variants or per_context or cfg2_full" > gpurun_out/${TAG}_variants.log 2>&1 || { tail -30 gpurun_out/${TAG}_variants.log; exit 1; } ;;
    ab8) AB_ROUNDS=8 timeout -k 10 300 python bench.py --ab --steps 30 --no-cpu --no-host-path --no-delivery > gpurun_out/${TAG}_ab8.json 2> gpurun_out/${TAG}_ab8.err || exit 1 ;;
    ab) timeout -k 10 200 python bench.py --ab --steps 30 --no-cpu --no-host-path --no-delivery > gpurun_out/${TAG}_ab.json 2> gpurun_out/${TAG}_ab.err || exit 1 ;;
    bench) timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_cfg2.json 2> gpurun_out/${TAG}_cfg2.err || exit 1 ;;
    cfg3) timeout -k 10 240 python bench.py --workload cfg3 > gpurun_out/${TAG}_cfg3.json 2> gpurun_out/${TAG}_cfg3.err || exit 1 ;;
    cfg4) timeout -k 10 200 python bench.py --workload cfg4 --steps 50 > gpurun_out/${TAG}_cfg4.json 2> gpurun_out/${TAG}_cfg4.err || exit 1 ;;
    cfg5) timeout -k 10 200 python bench.py --workload cfg5 --steps 50 > gpurun_out/${TAG}_cfg5.json 2> gpurun_out/${TAG}_cfg5.err || exit 1 ;;
    filesums) timeout -k 10 300 python bench.py --workload filesums > gpurun_out/${TAG}_filesums.json 2> gpurun_out/${TAG}_filesums.err || exit 1 ;;
    receive) timeout -k 10 300 python bench.py --workload receive > gpurun_out/${TAG}_receive.json 2> gpurun_out/${TAG}_receive.err || exit 1 ;;
    cfg4s) timeout -k 10 400 python bench.py --workload cfg4-sender --steps 10 --cpu-seconds 5 > gpurun_out/${TAG}_cfg4s.json 2> gpurun_out/${TAG}_cfg4s.err || exit 1 ;;
    sqrt) SWEEP_SQRT=1 SWEEP_ONLY=automatic timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${TAG}_sqrt.jsonl 2> gpurun_out/${TAG}_sqrt.err || exit 1 ;;
    prof_cfg4s) PASSES="FETCH_SIZE;WRITE_SIZE" bash tools/profile_kernel.sh ${TAG}_cfg4s search_small --workload cfg4-sender --steps 3 --warmup 1 --no-cpu || exit 1 ;;
    prof_cfg2) bash tools/profile_kernel.sh ${TAG}_cfg2 block_sums --steps 20 --warmup 5 --no-cpu --no-host-path --no-delivery || exit 1 ;;
    prof_cfg3) PASSES="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE;FETCH_SIZE" bash tools/profile_kernel.sh ${TAG}_cfg3 roll --workload cfg3 --steps 2 --warmup 1 --cfg3-files 4 --no-cpu --no-host-path || exit 1 ;;
    prof_cfg4) PASSES="FETCH_SIZE;WRITE_SIZE" bash tools/profile_kernel.sh ${TAG}_cfg4 block_sums --workload cfg4 --steps 20 --no-cpu --no-host-path --no-delivery || exit 1 ;;
    prof_cfg5) PASSES="FETCH_SIZE;WRITE_SIZE" bash tools/profile_kernel.sh ${TAG}_cfg5 block_sums --workload cfg5 --steps 5 --warmup 2 --no-cpu || exit 1 ;;
    prof_filesums) PASSES="FETCH_SIZE;WRITE_SIZE" bash tools/profile_kernel.sh ${TAG}_filesums file_sums --workload filesums --no-cpu || exit 1 ;;
    *) echo "unknown step $S"; exit 2 ;;
  esac
done
echo "[$TAG] done $(date +%T)"
