# Copy a round profile from gpurun_out/ into profiles/ (tracked):
#   bash tools/save_round_profile.sh <tag>
# needs gpurun_out/prof_<tag>/ (tools/profile_round.sh) and gpurun_out/bench_<tag>.json (tools/gpu_round.sh bench)
set -e
TAG=$1; P=gpurun_out/prof_$TAG
cp $P/trace/bench_kernel_stats.csv profiles/${TAG}_bench_kernel_stats.csv
python3 tools/stats_table.py $P/trace/bench_kernel_stats.csv --top 40 \
  --title "rocprofv3 --kernel-trace --stats -- python3 bench.py (defaults), tools/profile_round.sh $TAG" > profiles/${TAG}_bench_kernel_stats.txt
tail -1 $P/bench_line.txt > profiles/${TAG}_bench_line_under_rocprof.json
cp $P/pmc_traffic.json profiles/${TAG}_pmc_traffic.json
[ -f gpurun_out/bench_$TAG.json ] && tail -1 gpurun_out/bench_$TAG.json > profiles/${TAG}_bench_line.json
ls -la profiles/${TAG}_*
