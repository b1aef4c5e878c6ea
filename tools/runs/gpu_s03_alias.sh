# Finalize ranking keys aliased onto the list LDS (fewer bytes per workgroup): old vs new, then the final check.
set -e
mkdir -p gpurun_out/al
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for args in "2048 105542 1000" "131072 105542 100"; do
  for v in old alias old alias; do
    tag=$v.$(echo $args | tr ' ' _)
    timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/al/$tag -o run -- ./tools/pbin/probe_$v $args > gpurun_out/al/$tag.log 2>&1
    f=$(find gpurun_out/al/$tag -name '*kernel_stats.csv' | head -1)
    echo "== $v [$args] $(grep nq= gpurun_out/al/$tag.log | tail -1) | $(grep top5 gpurun_out/al/$tag.log)"
    python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if 'finalize' in n: print('   ', n[:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
    rm -rf gpurun_out/al/$tag
  done
done
bash tools/runs/gpu_s03_final.sh
