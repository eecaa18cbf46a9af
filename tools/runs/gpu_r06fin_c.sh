# Final evidence pass, part C: rocprofv3 traces + PMC passes per workload,
# summarized on the box; raw counter CSVs removed so the output stays small.
set -o pipefail
cd $GRAFT_REPO_ROOT
S=gpurun_out/r06fin_summ
mkdir -p $S
bash tools/gpu_run.sh r06fin prof_cfg2 prof_cfg3 prof_cfg4 prof_cfg4s prof_cfg5 prof_filesums || exit 2
python3 tools/summarize_profile.py r06fin_cfg2 --kernel block_sums --outdir $S --timed 100 > /dev/null || exit 3
python3 tools/summarize_profile.py r06fin_cfg3 --kernel roll_packed --outdir $S > /dev/null || exit 3
python3 tools/summarize_profile.py r06fin_cfg4 --kernel block_sums --outdir $S --traffic-key block_sums_kernel_cfg4_bytes_per_launch > /dev/null || exit 3
python3 tools/summarize_profile.py r06fin_cfg4s --kernel search_small --outdir $S --no-traffic > /dev/null || exit 3
python3 tools/summarize_profile.py r06fin_cfg5 --kernel block_sums --outdir $S --traffic-key block_sums_kernel_cfg5_bytes_per_launch > /dev/null || exit 3
python3 tools/summarize_profile.py r06fin_filesums --kernel file_sums --outdir $S --traffic-key file_sums_kernel_cfg4set_bytes_per_launch > /dev/null || exit 3
for d in gpurun_out/prof_r06fin_*; do
  t=$(basename $d)
  cp $d/trace/*kernel_stats.csv $S/${t}_kernel_stats.csv 2>/dev/null
  rm -rf $d
done
du -sh gpurun_out
