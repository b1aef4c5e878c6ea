# Finalize rescoring variants (LDS-staged rows), then GPU suite + smoke + pair A/B.
set -e
mkdir -p gpurun_out/finp
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in f0 f16b2 f16b1 f32b1 f32b2 f8b2; do
  timeout -k 10 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/finp/$v -o run -- ./tools/pbin/probe_$v 131072 > gpurun_out/finp/$v.log 2>&1
  f=$(find gpurun_out/finp/$v -name '*kernel_stats.csv' | head -1)
  echo "== $v $(grep nq= gpurun_out/finp/$v.log | tail -1) | $(grep top5 gpurun_out/finp/$v.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
  n=r['Name']
  if 'scan_kernel<128>' in n or 'finalize' in n or 'fallback' in n: print('   ', n[:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"
done
bash tools/runs/gpu_s03_suite_pair_ab.sh
