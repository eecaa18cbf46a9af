#!/bin/bash
# cfg3: CUs left to the confirmation (RSG_CONFIRM_CUS) with the default kernels, two rounds
mkdir -p gpurun_out
for r in 1 2; do
  for k in 0 32 40 48 64; do
    RSG_CONFIRM_CUS=$k timeout -k 10 200 python bench.py --workload cfg3 --no-cpu --no-host-path > gpurun_out/ab2_r${r}_k$k.json 2> gpurun_out/ab2_r${r}_k$k.err || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
RSG_CONFIRM_CUS=40 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl40 -o tl -- python3 bench.py --workload cfg3 --cfg3-files 4 --steps 1 --no-cpu --no-host-path > gpurun_out/ab2_tl.log 2>&1
