set -o pipefail
cd $GRAFT_REPO_ROOT
T=r05ay
bash tools/gpu_run.sh $T tests smoke bench || exit 1
timeout -k 10 300 python tools/pack_align_ab.py > gpurun_out/${T}_pack_align.jsonl 2> gpurun_out/${T}_pack_align.err || exit 4
