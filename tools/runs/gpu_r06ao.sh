# On-the-lines block lengths: variant 4 (the rule's choice) against the line-window kernel (7) and staged (1)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SWEEP_SQRT=1,9,64 SWEEP_ONLY=automatic,staged_seg128,lines,staged SWEEP_ROUNDS=2 timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/r06ao_sqrt_lines.jsonl 2> gpurun_out/r06ao_sqrt_lines.err || exit 1
SWEEP_BLENS=1024,2048,4096,8192 SWEEP_ONLY=automatic,staged_seg128,lines,staged SWEEP_ROUNDS=2 timeout -k 10 300 python tools/blocklen_sweep.py > gpurun_out/r06ao_blens_lines.jsonl 2> gpurun_out/r06ao_blens_lines.err || exit 1
python -c "
import json
for f in ('gpurun_out/r06ao_sqrt_lines.jsonl','gpurun_out/r06ao_blens_lines.jsonl'):
    for l in open(f):
        d=json.loads(l); print(d['block_len'], d['file_bytes'], {k:v['kernel_ms'] for k,v in d['variants'].items()})
"
