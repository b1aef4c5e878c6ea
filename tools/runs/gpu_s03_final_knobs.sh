# Finalize knobs (list staging size, two-row rescoring), then the round bench + profile.
set -e
mkdir -p gpurun_out/fink
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in base st lf768 lf640 lf512 r2c8 r2c16 r2c8lf768; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fink/$v -o run -- ./tools/pbin/probe_$v 131072 > gpurun_out/fink/$v.log 2>&1
  f=$(find gpurun_out/fink/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v $(grep nq= gpurun_out/fink/$v.log | tail -1) | $(grep top5 gpurun_out/fink/$v.log) $(grep 'list entries' gpurun_out/fink/$v.log | tail -1)"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if 'scan_kernel<128>' in n or 'finalize' in n or 'fallback' in n: print('   ', n[:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
timeout -k 10 500 python -u bench.py > gpurun_out/bench_r03x.json 2> gpurun_out/bench_r03x.err || { tail -30 gpurun_out/bench_r03x.err; exit 1; }
cat gpurun_out/bench_r03x.json
bash tools/profile_round.sh r03x
