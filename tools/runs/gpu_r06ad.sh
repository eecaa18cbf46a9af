set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06ad
mkdir -p gpurun_out
RSG_TIMING=1 timeout -k 10 300 python bench.py --workload cfg3 --no-host-path --no-cpu --steps 2 --warmup 1 > gpurun_out/${T}_cfg3.json 2> gpurun_out/${T}_cfg3.err || { tail -20 gpurun_out/${T}_cfg3.err; exit 6; }
grep "\[rsg\]" gpurun_out/${T}_cfg3.err | tail -150 > gpurun_out/${T}_phases.txt
wc -l gpurun_out/${T}_phases.txt
