# rocprofv3 evidence of the final code: traces + PMC passes per workload,
# summarized on the box (gpurun_out/<tag>_summ/: summaries, traffic.json,
# counters.json), raw counter CSVs removed so the output stays small.
set -o pipefail
cd $GRAFT_REPO_ROOT
S=gpurun_out/r05z_summ
mkdir -p $S
bash tools/gpu_run.sh r05z prof_cfg2 prof_cfg3 prof_cfg4 prof_cfg5 prof_filesums || exit 2
python3 tools/summarize_profile.py r05z_cfg2 --kernel block_sums --outdir $S --timed 100 > /dev/null || exit 3
python3 tools/summarize_profile.py r05z_cfg3 --kernel roll_packed --outdir $S > /dev/null || exit 3
python3 tools/summarize_profile.py r05z_cfg4 --kernel block_sums --outdir $S --traffic-key block_sums_kernel_cfg4_bytes_per_launch > /dev/null || exit 3
python3 tools/summarize_profile.py r05z_cfg5 --kernel block_sums --outdir $S --traffic-key block_sums_kernel_cfg5_bytes_per_launch > /dev/null || exit 3
python3 tools/summarize_profile.py r05z_filesums --kernel file_sums --outdir $S --traffic-key file_sums_kernel_cfg4set_bytes_per_launch > /dev/null || exit 3
for d in gpurun_out/prof_r05z_*; do
  t=$(basename $d)
  cp $d/trace/*kernel_stats.csv $S/${t}_kernel_stats.csv 2>/dev/null
  cp $d/trace.log $S/${t}_trace.log 2>/dev/null
  rm -rf $d
done
du -sh gpurun_out
