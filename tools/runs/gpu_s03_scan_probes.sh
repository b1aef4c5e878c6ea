# Index scan probes: per-variant scan_kernel time (rocprofv3 stats) at one 131k-query chunk.
set -e
mkdir -p gpurun_out/scanp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base noresc p2 p1 prio1 prio2 noins noinsprio1 p2prio2; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/scanp/$v -o run -- ./tools/pbin/probe_$v 131072 > gpurun_out/scanp/$v.log 2>&1
  f=$(find gpurun_out/scanp/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v $(grep -v amdgpu.ids gpurun_out/scanp/$v.log | grep nq= | head -1)"
  python3 -c "
import csv,sys
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if 'scan_kernel<128>' in n or 'finalize' in n or 'sample_kernel<128>' in n or 'fallback' in n: print('   ', n[:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
