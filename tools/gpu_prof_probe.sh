# Kernel-trace stats of probe binaries (tools/pbin) on the GPU box.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
rm -rf $R/gpurun_out/prof_probe
for v in ${VARIANTS:-stats}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_probe -o $v -- $R/tools/pbin/probe_$v ${NQ:-131072} > /dev/null 2>&1
done
