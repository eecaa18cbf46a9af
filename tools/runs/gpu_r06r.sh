set -o pipefail
cd $GRAFT_REPO_ROOT
T=r06r
mkdir -p gpurun_out
timeout -k 10 200 python tools/confirm_probe.py 32768 64 256 2368 4736 23515 > gpurun_out/${T}_probe.jsonl 2> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 3; }
cat gpurun_out/${T}_probe.jsonl
timeout -k 10 200 python tools/confirm_probe.py 32767 2368 > gpurun_out/${T}_probe2.jsonl 2>> gpurun_out/${T}.err || { tail -20 gpurun_out/${T}.err; exit 4; }
cat gpurun_out/${T}_probe2.jsonl
