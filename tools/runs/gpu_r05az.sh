set -o pipefail
cd $GRAFT_REPO_ROOT
T=r05az
bash tools/gpu_run.sh $T tests smoke bench || exit 1
timeout -k 10 300 python tools/pack_align_ab.py > gpurun_out/${T}_pack_align.jsonl 2> gpurun_out/${T}_pack_align.err || exit 4
SWEEP_ONLY=automatic timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep_pow2.jsonl 2> gpurun_out/${T}_sweep_pow2.err || exit 5
SWEEP_BLENS=1000,1224,2176,4000,4096,6144,9000 SWEEP_ONLY=automatic timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/${T}_sweep_real.jsonl 2> gpurun_out/${T}_sweep_real.err || exit 6
