set -o pipefail
mkdir -p gpurun_out/prof_e
cd /tmp && export TMPDIR=/tmp
for n in iprobe_base iprobe2_base; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_e/$n -o run -- $GRAFT_REPO_ROOT/tools/pbin/$n 131072 > $GRAFT_REPO_ROOT/gpurun_out/prof_e/$n.log 2>&1 || exit 1
done
cd $GRAFT_REPO_ROOT
for n in iprobe_base iprobe2_base; do echo "== $n"; f=$(find gpurun_out/prof_e/$n -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 $f | head -12; done
