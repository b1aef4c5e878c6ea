set -e
mkdir -p gpurun_out
O=gpurun_out/probe.log
: > $O
timeout -k 10 120 ./tools/pbin/probe_stats 131072 >> $O 2>&1
timeout -k 10 120 ./tools/pbin/probe_noins 131072 >> $O 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_probe -o noins -- $GRAFT_REPO_ROOT/tools/pbin/probe_noins 131072 >> $GRAFT_REPO_ROOT/$O 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_probe -o stats -- $GRAFT_REPO_ROOT/tools/pbin/probe_stats 131072 >> $GRAFT_REPO_ROOT/$O 2>&1
