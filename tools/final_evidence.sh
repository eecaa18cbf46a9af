#!/bin/bash
# Round-end evidence on one MI355X: GPU parity suite, smoke, every bench
# workload (tools/gpu_run.sh steps), then the rocprofv3 kernel trace + PMC
# passes of cfg2 / cfg3 / cfg4 / cfg5 / filesums, summarized on the box into
# gpurun_out/<tag>_summ/ (summaries, traffic.json, counters.json, kernel
# stats) with the raw CSVs removed, so the call's output stays small.
# Usage: tools/final_evidence.sh <tag>   (copy <tag>_summ/* into profiles/)
set -o pipefail
T=${1:-r05z}
S=gpurun_out/${T}_summ
mkdir -p $S
bash tools/gpu_run.sh $T tests smoke bench cfg3 cfg4 cfg5 filesums receive || exit 1
bash tools/gpu_run.sh $T prof_cfg2 prof_cfg3 prof_cfg4 prof_cfg5 prof_filesums || exit 2
python3 tools/summarize_profile.py ${T}_cfg2 --kernel block_sums --outdir $S --timed 100 > /dev/null || exit 3
python3 tools/summarize_profile.py ${T}_cfg3 --kernel roll_packed --outdir $S > /dev/null || exit 3
python3 tools/summarize_profile.py ${T}_cfg4 --kernel block_sums --outdir $S --traffic-key block_sums_kernel_cfg4_bytes_per_launch > /dev/null || exit 3
python3 tools/summarize_profile.py ${T}_cfg5 --kernel block_sums --outdir $S --traffic-key block_sums_kernel_cfg5_bytes_per_launch > /dev/null || exit 3
python3 tools/summarize_profile.py ${T}_filesums --kernel file_sums --outdir $S --traffic-key file_sums_kernel_cfg4set_bytes_per_launch > /dev/null || exit 3
for d in gpurun_out/prof_${T}_*; do
  b=$(basename $d)
  cp $d/trace/*kernel_stats.csv $S/${b}_kernel_stats.csv 2>/dev/null
  rm -rf $d
done
echo "[$T] evidence in $S"
