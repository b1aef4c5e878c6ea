# Runner index point (2048 queries, k = 1000): split-count knobs.
set -e
mkdir -p gpurun_out/sp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base basest s32 s32st s64 s64st; do
  for args in "2048 105542 1000" "2048 105542 100"; do
    tag=$v.$(echo $args | tr ' ' _)
    timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sp/$tag -o run -- ./tools/pbin/probe_$v $args > gpurun_out/sp/$tag.log 2>&1
    f=$(find gpurun_out/sp/$tag -name '*kernel_stats.csv' | head -1)
    echo "== $v [$args] $(grep nq= gpurun_out/sp/$tag.log | tail -1) | $(grep top5 gpurun_out/sp/$tag.log) $(grep 'list entries' gpurun_out/sp/$tag.log | tail -1)"
    python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if any(x in n for x in ('scan_kernel<128>','sample_kernel<128>','finalize','fallback')): print('   ', n[:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
    rm -rf gpurun_out/sp/$tag
  done
done
